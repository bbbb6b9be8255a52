// Small HBM-bound kernels of the path:
//   nr_score_fwd/bwd      batched user x candidate scorer + log_softmax / sigmoid head
//                         (models/TwoTowerBaseModel.py:51-75, predict_fast :78-83 with a
//                         gathered news table)
//   nr_adam               Adam update, torch.optim.Adam semantics (utils/Manager.py:404-413,647)
//   nr_embedding_fwd/bwd  standalone word-embedding lookup and its padding_idx-aware
//                         scatter-add backward (models/Embeddings/BERT.py:39)
//   nr_colsum             column sums (bias gradients of the projections)
#include "common.h"
#include "../../include/newsrec_hip.h"

namespace {

// one workgroup (256 threads) per impression b; one wave per candidate dot product
__global__ __launch_bounds__(256) void score_fwd_kernel(const float* cdd, int64_t ldc, const int64_t* cdd_idx,
                                                        const float* user, int64_t ldu, int C, int H,
                                                        float scale, int mode, float* logits) {
  extern __shared__ float sc[];
  const int b = blockIdx.x, tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const float* u = user + (int64_t)b * ldu;
  for (int c = w; c < C; c += 4) {
    const int64_t row = cdd_idx ? cdd_idx[(int64_t)b * C + c] : (int64_t)b * C + c;
    const float* x = cdd + row * ldc;
    float s = 0.f;
    for (int d = lane; d < H; d += 64) s = fmaf(x[d], u[d], s);
    s = nr_wave_sum(s);
    if (lane == 0) sc[c] = s * scale;
  }
  __syncthreads();
  if (mode == NR_SCORE_LOG_SOFTMAX) {
    if (w == 0) {
      float mx = -INFINITY;
      for (int c = lane; c < C; c += 64) mx = fmaxf(mx, sc[c]);
      mx = nr_wave_max(mx);
      float sum = 0.f;
      for (int c = lane; c < C; c += 64) sum += __expf(sc[c] - mx);
      const float lse = mx + __logf(nr_wave_sum(sum));
      for (int c = lane; c < C; c += 64) logits[(int64_t)b * C + c] = sc[c] - lse;
    }
  } else {
    for (int c = tid; c < C; c += 256) {
      const float s = sc[c];
      logits[(int64_t)b * C + c] = mode == NR_SCORE_SIGMOID ? 1.f / (1.f + __expf(-s)) : s;
    }
  }
}

__global__ __launch_bounds__(256) void score_bwd_kernel(const float* cdd, int64_t ldc, const float* user,
                                                        int64_t ldu, const float* logits,
                                                        const float* dlogits, int C, int H, float scale,
                                                        int mode, float* dcdd, int64_t lddc, float* duser,
                                                        int64_t lddu) {
  extern __shared__ float ds[];
  const int b = blockIdx.x, tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  // d score
  if (w == 0) {
    if (mode == NR_SCORE_LOG_SOFTMAX) {
      float sg = 0.f;
      for (int c = lane; c < C; c += 64) sg += dlogits[(int64_t)b * C + c];
      sg = nr_wave_sum(sg);
      for (int c = lane; c < C; c += 64) {
        const int64_t o = (int64_t)b * C + c;
        ds[c] = (dlogits[o] - __expf(logits[o]) * sg) * scale;
      }
    } else {
      for (int c = lane; c < C; c += 64) {
        const int64_t o = (int64_t)b * C + c;
        const float y = logits[o];
        ds[c] = (mode == NR_SCORE_SIGMOID ? dlogits[o] * y * (1.f - y) : dlogits[o]) * scale;
      }
    }
  }
  __syncthreads();
  const float* u = user + (int64_t)b * ldu;
  for (int d = tid; d < H; d += 256) {
    float acc = 0.f;
    const float ud = u[d];
    for (int c = 0; c < C; ++c) {
      const float* x = cdd + ((int64_t)b * C + c) * ldc;
      acc = fmaf(ds[c], x[d], acc);
      dcdd[((int64_t)b * C + c) * lddc + d] = ds[c] * ud;
    }
    duser[(int64_t)b * lddu + d] = acc;
  }
}

// Training head + NLLLoss (Manager.py:641, torch.nn.NLLLoss(): reduction 'mean', ignore_index -100)
// in one launch: workgroup b forms the C scores of impression b (one wave per candidate dot product),
// their log-softmax, its loss term part[b] and its weight wt[b] (1 for a label in [0, C), 0 for the
// ignored label -100, NaN for any other label); the workgroup that arrives last (agent-scope release +
// ticket, acquire: cdna_hip_programming.md §6 Guideline 16's counter form) forms sum(part) / sum(wt)
// in a fixed order (deterministic: torch's weighted mean -- NaN when every label is ignored, as 0/0 --
// and NaN for an out-of-range label, where torch raises) and resets the ticket.  work[0] is the ticket
// (zero again on return), work[1] a sticky status: non-zero once a label outside [0, C) other than
// -100 was seen (read and cleared by the host, nr_score_nll_workspace's layout).
constexpr int64_t kIgnoreIndex = -100;

__global__ __launch_bounds__(1024) void score_nll_fwd_kernel(const float* cdd, int64_t ldc, const float* user,
                                                             int64_t ldu, const int64_t* label, int B, int C, int H,
                                                             float scale, float* logits, float* loss,
                                                             int32_t* work) {
  extern __shared__ float sc[];   // [C] scores
  __shared__ int last;
  const int b = blockIdx.x, tid = threadIdx.x, w = tid >> 6, lane = tid & 63, nw = blockDim.x >> 6;
  float* part = reinterpret_cast<float*>(work + 4);
  float* wt = part + B;
  const float* u = user + (int64_t)b * ldu;
  for (int c = w; c < C; c += nw) {
    const float* x = cdd + ((int64_t)b * C + c) * ldc;
    float s = 0.f;
    for (int d = lane; d < H; d += 64) s = fmaf(x[d], u[d], s);
    s = nr_wave_sum(s);
    if (lane == 0) sc[c] = s * scale;
  }
  __syncthreads();
  if (w == 0) {
    float mx = -INFINITY;
    for (int c = lane; c < C; c += 64) mx = fmaxf(mx, sc[c]);
    mx = nr_wave_max(mx);
    float sum = 0.f;
    for (int c = lane; c < C; c += 64) sum += __expf(sc[c] - mx);
    const float lse = mx + __logf(nr_wave_sum(sum));
    for (int c = lane; c < C; c += 64) logits[(int64_t)b * C + c] = sc[c] - lse;
    if (lane == 0) {
      const int64_t y = label[b];
      const bool ok = y >= 0 && y < C;
      part[b] = ok ? -(sc[y] - lse) : 0.f;
      wt[b] = ok ? 1.f : (y == kIgnoreIndex ? 0.f : __int_as_float(0x7fc00000));
      if (!ok && y != kIgnoreIndex) __hip_atomic_store(&work[1], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int ticket = atomicAdd(&work[0], 1);
    last = ticket == B - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (!last || w != 0) return;
  float s = 0.f, n = 0.f;   // fixed-order sums of the B terms and weights
  for (int r = lane; r < B; r += 64) {
    s += part[r];
    n += wt[r];
  }
  s = nr_wave_sum(s);
  n = nr_wave_sum(n);
  if (lane == 0) {
    loss[0] = s / n;
    __hip_atomic_store(&work[0], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Backward of score_nll_fwd_kernel: d logits = dlogits (optional) - dloss / n at the label (n = the
// labels in [0, C), counted by each workgroup; ignored labels get no term), then the log-softmax
// and dot-product backward (as score_bwd_kernel), one workgroup per impression.
__global__ __launch_bounds__(256) void score_nll_bwd_kernel(const float* cdd, int64_t ldc, const float* user,
                                                            int64_t ldu, const float* logits, const int64_t* label,
                                                            const float* dloss, const float* dlogits, int B, int C,
                                                            int H, float scale, float* dcdd, int64_t lddc,
                                                            float* duser, int64_t lddu) {
  extern __shared__ float ds[];
  const int b = blockIdx.x, tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  if (w == 0) {
    const int64_t y = label[b];
    float gl = 0.f;
    if (dloss) {
      float n = 0.f;
      for (int r = lane; r < B; r += 64) {
        const int64_t yr = label[r];
        n += (yr >= 0 && yr < C) ? 1.f : 0.f;
      }
      gl = -dloss[0] / nr_wave_sum(n);
    }
    float sg = 0.f;
    for (int c = lane; c < C; c += 64) {
      const int64_t o = (int64_t)b * C + c;
      sg += (dlogits ? dlogits[o] : 0.f) + (c == y ? gl : 0.f);
    }
    sg = nr_wave_sum(sg);
    for (int c = lane; c < C; c += 64) {
      const int64_t o = (int64_t)b * C + c;
      const float g = (dlogits ? dlogits[o] : 0.f) + (c == y ? gl : 0.f);
      ds[c] = (g - __expf(logits[o]) * sg) * scale;
    }
  }
  __syncthreads();
  const float* u = user + (int64_t)b * ldu;
  for (int d = tid; d < H; d += 256) {
    float acc = 0.f;
    const float ud = u[d];
    for (int c = 0; c < C; ++c) {
      const float* x = cdd + ((int64_t)b * C + c) * ldc;
      acc = fmaf(ds[c], x[d], acc);
      dcdd[((int64_t)b * C + c) * lddc + d] = ds[c] * ud;
    }
    duser[(int64_t)b * lddu + d] = acc;
  }
}

// torch.optim.Adam (foreach=False, maximize=False, amsgrad=False) per element:
//   g += wd * p;  m = lerp(m, g, 1 - b1);  v = b2 v + (1 - b2) g²
//   p -= (lr / bc1) * m / (sqrt(v) / sqrt(bc2) + eps)
// step_dev (graph replays): the step count lives on the device and the bias corrections are
// formed per workgroup in double, as torch forms them in Python floats.
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                   float step, float b1, float b2, float eps,
                                                   float bc2_sqrt, float wd, float gscale,
                                                   const int64_t* __restrict__ step_dev, float lr) {
  if (step_dev) {
    __shared__ float sc[2];
    if (threadIdx.x == 0) {
      const double t = (double)*step_dev;
      const double bc1 = 1.0 - pow((double)b1, t), bc2 = 1.0 - pow((double)b2, t);
      sc[0] = (float)((double)lr / bc1);
      sc[1] = (float)sqrt(bc2);
    }
    __syncthreads();
    step = sc[0];
    bc2_sqrt = sc[1];
  }
  const int64_t n4 = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 pp = reinterpret_cast<float4*>(p)[i];
    float4 gg = reinterpret_cast<const float4*>(g)[i];
    float4 mm = reinterpret_cast<float4*>(m)[i];
    float4 vv = reinterpret_cast<float4*>(v)[i];
#define NR_ADAM1(c)                                            \
    {                                                          \
      float gc = gg.c * gscale;                                \
      if (wd != 0.f) gc = fmaf(wd, pp.c, gc);                  \
      mm.c = fmaf(1.f - b1, gc - mm.c, mm.c);                  \
      vv.c = fmaf(vv.c, b2, (1.f - b2) * gc * gc);             \
      const float den = sqrtf(vv.c) / bc2_sqrt + eps;          \
      pp.c = fmaf(-step, mm.c / den, pp.c);                    \
    }
    NR_ADAM1(x) NR_ADAM1(y) NR_ADAM1(z) NR_ADAM1(w)
    reinterpret_cast<float4*>(p)[i] = pp;
    reinterpret_cast<float4*>(m)[i] = mm;
    reinterpret_cast<float4*>(v)[i] = vv;
  }
  for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float gc = g[i] * gscale;
    if (wd != 0.f) gc = fmaf(wd, p[i], gc);
    m[i] = fmaf(1.f - b1, gc - m[i], m[i]);
    v[i] = fmaf(v[i], b2, (1.f - b2) * gc * gc);
    const float den = sqrtf(v[i]) / bc2_sqrt + eps;
    p[i] = fmaf(-step, m[i] / den, p[i]);
  }
#undef NR_ADAM1
}

// ---- multi-tensor Adam: up to kAdamMulti tensors per launch, their descriptors passed by value
// (graph-capturable: no device-side pointer table), blocks assigned to tensors by a prefix sum
constexpr int kAdamMulti = 32;   // the descriptors travel as kernel arguments (< 4 KB)
constexpr int kAdamChunk = 4096;   // elements per block (256 threads x 4 float4)

struct AdamEntry {
  float* p; const float* g; float* m; float* v;
  int64_t n;
  int64_t* step_dev;         // device step count (graph replays) or null
  const float* lr_dev;       // device learning rate (a scheduler updates it between replays) or null
  float step_size;           // lr / (1 - beta1^t) when neither is on the device
  float bc2_sqrt;            // sqrt(1 - beta2^t) when step_dev is null
  float lr;
  int64_t step;              // host step count
  const uint8_t* rt;         // optional per-row "gradient non-zero" flags (rows of rlen elements)
  int64_t rlen;
};

struct AdamMulti {
  AdamEntry e[kAdamMulti];
  int32_t blk_off[kAdamMulti + 1];
  int count;
  int32_t* ticket;   // non-null: the launch advances the device step counts itself (nr_adam_multi_step)
  float b1, b2, eps, wd, gscale;
};

__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, float b1, float b2, float eps,
                                          float wd, float gscale, float step, float bc2_sqrt) {
  float gc = g * gscale;
  if (wd != 0.f) gc = fmaf(wd, p, gc);
  m = fmaf(1.f - b1, gc - m, m);
  v = fmaf(v, b2, (1.f - b2) * gc * gc);
  const float den = sqrtf(v) / bc2_sqrt + eps;
  p = fmaf(-step, m / den, p);
}

// p / m / v are written with nontemporal stores (streamed out, not kept in the L2s): same-box A/B on
// the NRMS parameter set (24.6 M, 690 MB per step), profiles/r04_h_adam_ab.json: 134 -> 109 us; making
// the loads nontemporal too measured 120 us
typedef float adam_f4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 adam_ld(const float* base, int64_t i) { return reinterpret_cast<const float4*>(base)[i]; }
__device__ __forceinline__ void adam_st(float* base, int64_t i, float4 v) {
  __builtin_nontemporal_store((adam_f4){v.x, v.y, v.z, v.w}, reinterpret_cast<adam_f4*>(base) + i);
}

__global__ __launch_bounds__(256) void adam_multi_kernel(AdamMulti a) {
  const int b = blockIdx.x;
  int t = 0;
  while (t + 1 < a.count && b >= a.blk_off[t + 1]) ++t;
  const AdamEntry& e = a.e[t];
  float step = e.step_size, bc2_sqrt = e.bc2_sqrt;
  // device step count / learning rate: the bias corrections in double precision, by ONE lane of the
  // workgroup (the other 255 would repeat two pow() calls each), after the thread's loads are issued
  const bool dev_sched = e.step_dev || e.lr_dev;
  __shared__ float s_sched[2];
  auto dev_schedule = [&]() {
    if (threadIdx.x == 0) {
      // with a ticket the device count is the one before this step: this step is count + 1
      const double st = e.step_dev ? (double)*e.step_dev + (a.ticket ? 1.0 : 0.0) : (double)e.step;
      const double lr = e.lr_dev ? (double)*e.lr_dev : (double)e.lr;
      s_sched[0] = (float)(lr / (1.0 - pow((double)a.b1, st)));
      s_sched[1] = (float)sqrt(1.0 - pow((double)a.b2, st));
    }
    __syncthreads();
    step = s_sched[0];
    bc2_sqrt = s_sched[1];
  };
  const int64_t base = (int64_t)(b - a.blk_off[t]) * kAdamChunk;
  const int64_t end = base + kAdamChunk < e.n ? base + kAdamChunk : e.n;
  const bool vec = ((reinterpret_cast<uintptr_t>(e.p) | reinterpret_cast<uintptr_t>(e.g) |
                     reinterpret_cast<uintptr_t>(e.m) | reinterpret_cast<uintptr_t>(e.v)) & 15) == 0;
  if (!(vec && end - base == kAdamChunk) && dev_sched) dev_schedule();   // (workgroup-uniform branch)
  if (vec && end - base == kAdamChunk) {
    // all sixteen float4 loads of the thread in flight before the first store (the four tensors
    // are distinct allocations; without the explicit order the stores of one float4 would have
    // to land before the next one's loads could be issued)
    float4 pp[4], gg[4], mm[4], vv[4];
    if (e.rt && e.n <= (int64_t)0x1fffffff) {
      // rows flagged untouched hold zeros: skip their gradient read (a float4 that reaches into a
      // touched row is read whole -- the untouched part reads as the zeros it holds).  The float4
      // spans rows (4i) / rlen .. (4i + 3) / rlen (up to four when rows are shorter than 4).  All
      // the thread's flags first, then the gradient through a buffer descriptor: a skipped float4
      // gets an out-of-range offset, which the range check answers with zeros without a memory
      // access -- no branch around the load, no flag -> load round trip per float4
      bool rd[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t i = base / 4 + u * 256 + threadIdx.x;
        const int64_t r0 = (4 * i) / e.rlen, r1 = (4 * i + 3) / e.rlen;   // (clamped: no branch, one batch)
        rd[u] = ((uint32_t)e.rt[r0] | (uint32_t)e.rt[r0 + 1 < r1 ? r0 + 1 : r1] |
                 (uint32_t)e.rt[r0 + 2 < r1 ? r0 + 2 : r1] | (uint32_t)e.rt[r1]) != 0;
      }
      const auto grs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(e.g), 0, (int)(e.n * 4), 0x00020000);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t i = base / 4 + u * 256 + threadIdx.x;
        pp[u] = adam_ld(e.p, i);
        const uint32_t off = rd[u] ? (uint32_t)(i * 16) : 0x80000000u;
        gg[u] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(grs, (int)off, 0, 0));
        mm[u] = adam_ld(e.m, i);
        vv[u] = adam_ld(e.v, i);
      }
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t i = base / 4 + u * 256 + threadIdx.x;
        pp[u] = adam_ld(e.p, i);
        bool rd = !e.rt;   // (a gradient over 2^29 elements with row flags: the per-float4 test)
        if (!rd)
          for (int64_t r = (4 * i) / e.rlen; r <= (4 * i + 3) / e.rlen && !rd; ++r) rd = e.rt[r] != 0;
        gg[u] = rd ? adam_ld(e.g, i) : make_float4(0.f, 0.f, 0.f, 0.f);
        mm[u] = adam_ld(e.m, i);
        vv[u] = adam_ld(e.v, i);
      }
    }
    if (dev_sched) dev_schedule();   // while the loads are in flight
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t i = base / 4 + u * 256 + threadIdx.x;
      adam_elem(pp[u].x, gg[u].x, mm[u].x, vv[u].x, a.b1, a.b2, a.eps, a.wd, a.gscale, step, bc2_sqrt);
      adam_elem(pp[u].y, gg[u].y, mm[u].y, vv[u].y, a.b1, a.b2, a.eps, a.wd, a.gscale, step, bc2_sqrt);
      adam_elem(pp[u].z, gg[u].z, mm[u].z, vv[u].z, a.b1, a.b2, a.eps, a.wd, a.gscale, step, bc2_sqrt);
      adam_elem(pp[u].w, gg[u].w, mm[u].w, vv[u].w, a.b1, a.b2, a.eps, a.wd, a.gscale, step, bc2_sqrt);
      adam_st(e.p, i, pp[u]);
      adam_st(e.m, i, mm[u]);
      adam_st(e.v, i, vv[u]);
    }
  } else {
    for (int64_t i = base + threadIdx.x; i < end; i += 256) {
      float pp = e.p[i], mm = e.m[i], vv = e.v[i];
      const float gv = (!e.rt || e.rt[i / e.rlen]) ? e.g[i] : 0.f;
      adam_elem(pp, gv, mm, vv, a.b1, a.b2, a.eps, a.wd, a.gscale, step, bc2_sqrt);
      e.p[i] = pp;
      e.m[i] = mm;
      e.v[i] = vv;
    }
  }
  if (a.ticket) {
    // every thread read its tensor's count at the top; the workgroup that finishes last advances
    // the counts of this launch's tensors for the next step and resets the ticket
    __syncthreads();
    if (threadIdx.x == 0 && atomicAdd(a.ticket, 1) == (int)gridDim.x - 1) {
      for (int t2 = 0; t2 < a.count; ++t2)
        if (a.e[t2].step_dev) atomicAdd(reinterpret_cast<unsigned long long*>(a.e[t2].step_dev), 1ull);
      __hip_atomic_store(a.ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// one wave per output row, float4 along E
__global__ __launch_bounds__(256) void embedding_fwd_kernel(const float* table, int64_t E, const int64_t* idx,
                                                            int64_t n, float* out) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n) return;
  const float4* src = reinterpret_cast<const float4*>(table + idx[row] * E);
  float4* dst = reinterpret_cast<float4*>(out + row * E);
  for (int64_t c = lane; c < E / 4; c += 64) dst[c] = src[c];
}

__global__ __launch_bounds__(256) void embedding_bwd_kernel(const float* dout, int64_t E, const int64_t* idx,
                                                            int64_t n, int64_t pad, float* dtable) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n) return;
  const int64_t t = idx[row];
  if (t == pad) return;
  for (int64_t c = lane; c < E; c += 64) atomicAdd(&dtable[t * E + c], dout[row * E + c]);
}

// Row-sparse gradient rows added in a FIXED order (nr_rows_add_ordered): the wave of an id's first
// occurrence sums every row j >= i of that id in ascending j and adds the sum to its table row; the
// waves of later occurrences do nothing.  No atomics, so duplicate ids (LSTUR's dropped user ids all
// land on row 0, RNN.py:100-101) give the same bits on every run and every rank.  A wave scans the
// ids in chunks of 64 (one ballot per chunk): O(n^2 / 64) id reads, for the few rows a row-sparse
// table receives per step (B per rank, B x world in the data-parallel exchange).
__global__ __launch_bounds__(256) void rows_add_ordered_kernel(const float* __restrict__ dout, int64_t ldo,
                                                               int64_t V, int64_t E, const int64_t* __restrict__ idx,
                                                               int64_t n, int64_t pad, float* __restrict__ dtable,
                                                               int64_t ldt) {
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= n) return;
  const int64_t t = idx[i];
  if (t == pad || t < 0 || t >= V) return;   // out-of-range ids are dropped, never written
  for (int64_t j0 = 0; j0 < i; j0 += 64) {   // an earlier occurrence owns the row
    const int64_t j = j0 + lane;
    if (__ballot(j < i && idx[j] == t) != 0ull) return;
  }
  for (int64_t c0 = 0; c0 < E; c0 += 64) {   // wave-uniform trip counts: every lane takes part in each ballot
    const int64_t c = c0 + lane;
    float s = 0.f;
    for (int64_t j0 = i; j0 < n; j0 += 64) {
      const int64_t j = j0 + lane;
      unsigned long long m = __ballot(j < n && idx[j] == t);
      while (m) {   // ascending j: the fixed summation order
        const int b = __builtin_ctzll(m);
        m &= m - 1;
        if (c < E) s += dout[(j0 + b) * ldo + c];
      }
    }
    if (c < E) dtable[t * ldt + c] += s;
  }
}

// XSoftmax (models/Modules/Attention.py:56-80) along rows of `cols` values, one wave per row:
// masked entries -> -inf, softmax, masked entries set to exactly 0 (a fully masked row is all zero);
// the backward is _softmax_backward_data: dx = y (dy - Σ dy y).
__global__ __launch_bounds__(256) void xsoftmax_fwd_kernel(const float* __restrict__ x, const void* __restrict__ mask,
                                                           int mdt, int64_t rows, int64_t cols,
                                                           float* __restrict__ out) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  const float* xr = x + r * cols;
  float mx = -INFINITY;
  for (int64_t c = lane; c < cols; c += 64)
    if (nr_mask_at(mask, mdt, r * cols + c)) mx = fmaxf(mx, xr[c]);
  mx = nr_wave_max(mx);
  float s = 0.f;
  for (int64_t c = lane; c < cols; c += 64)
    if (nr_mask_at(mask, mdt, r * cols + c)) s += __expf(xr[c] - mx);
  s = nr_wave_sum(s);
  const float inv = s > 0.f ? 1.f / s : 0.f;   // no unmasked entry: the row is all zero
  for (int64_t c = lane; c < cols; c += 64)
    out[r * cols + c] = nr_mask_at(mask, mdt, r * cols + c) ? __expf(xr[c] - mx) * inv : 0.f;
}

__global__ __launch_bounds__(256) void xsoftmax_bwd_kernel(const float* __restrict__ y, const float* __restrict__ dy,
                                                           int64_t rows, int64_t cols, float* __restrict__ dx) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  float s = 0.f;
  for (int64_t c = lane; c < cols; c += 64) s += dy[r * cols + c] * y[r * cols + c];
  s = nr_wave_sum(s);
  for (int64_t c = lane; c < cols; c += 64) dx[r * cols + c] = y[r * cols + c] * (dy[r * cols + c] - s);
}

// dst[i] = src[idx[i]] rows of `cols` floats (any width; float4 when the rows allow), one wave per row:
// the fast-eval history gather (the news table rows of each history slot, Manager.py:516).
__global__ __launch_bounds__(256) void gather_rows_kernel(const float* __restrict__ src, int64_t lds,
                                                          const int64_t* __restrict__ idx, int64_t n, int64_t cols,
                                                          float* __restrict__ dst, int64_t ldd, int vec4) {
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= n) return;
  const float* s = src + idx[i] * lds;
  float* d = dst + i * ldd;
  if (vec4) {
    for (int64_t c = lane; c < cols / 4; c += 64)
      reinterpret_cast<float4*>(d)[c] = reinterpret_cast<const float4*>(s)[c];
  } else {
    for (int64_t c = lane; c < cols; c += 64) d[c] = s[c];
  }
}

// dst[c][r] = src[r][c]: 64 x 64 tiles through LDS (row pad of one float: the column reads are
// conflict-free), coalesced float reads and writes.  The NRMS table dgrad's k-contiguous weight.
__global__ __launch_bounds__(256) void transpose_kernel(const float* __restrict__ src, int64_t lds, int64_t rows,
                                                        int64_t cols, float* __restrict__ dst, int64_t ldd) {
  __shared__ float t[64][65];
  const int64_t r0 = (int64_t)blockIdx.y * 64, c0 = (int64_t)blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int i = ty; i < 64; i += 4) {
    const int64_t r = r0 + i, c = c0 + tx;
    t[i][tx] = r < rows && c < cols ? src[r * lds + c] : 0.f;
  }
  __syncthreads();
  for (int i = ty; i < 64; i += 4) {
    const int64_t c = c0 + i, r = r0 + tx;
    if (c < cols && r < rows) dst[c * ldd + r] = t[tx][i];
  }
}

// Column sums, deterministic two-pass: pass 1 = one block per (64-column chunk, row block), each of
// its 4 waves strides the block's rows with its 64 lanes on 64 consecutive columns (256-B row
// segments, 8 loads in flight), the waves combine in LDS and store the block's partial row; pass 2
// sums the partials per column in row-block order.  No atomics: a few thousand blocks adding into
// the same H addresses serialise on the L2 (the old one-pass form ran at ~1 TB/s on [52800, 150]).
constexpr int kColsumBlocks = 1024;

// tick (nr_colsum_ws): per 64-column chunk arrival counters, zero on entry; the chunk's last
// workgroup to arrive sums the chunk's partial rows in row-block order and resets its counter, so the
// final pass needs no launch of its own (cdna_hip_programming.md §6 Guideline 16's counter form with
// write-through partials: sc1 stores need no release fence -- the storing wave's vmcnt drain, the
// barrier, lane 0's agent-scope ticket; the last arriver's acquire, then plain loads)
__global__ __launch_bounds__(256) void colsum_part_kernel(const float* __restrict__ x, int64_t ldx, int64_t rows,
                                                          int64_t cols, int64_t rb_rows, float* __restrict__ part,
                                                          int32_t* __restrict__ tick, float* __restrict__ out) {
  __shared__ float red[4][64];
  __shared__ int last;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t c = (int64_t)blockIdx.x * 64 + lane;
  const int64_t r0 = (int64_t)blockIdx.y * rb_rows;
  const int64_t r1 = r0 + rb_rows < rows ? r0 + rb_rows : rows;
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c < cols) {
    int64_t r = r0 + w;
    const float* p = x + r * ldx + c;
    for (; r + 28 < r1; r += 32, p += 32 * ldx) {
#pragma unroll
      for (int u = 0; u < 8; ++u) a[u] += p[4 * u * ldx];
    }
    for (; r < r1; r += 4, p += 4 * ldx) a[0] += *p;
  }
  red[w][lane] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  __syncthreads();
  if (!tick) {
    if (w == 0 && c < cols) part[(int64_t)blockIdx.y * cols + c] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
    return;
  }
  if (w == 0 && c < cols)
    __hip_atomic_store(&part[(int64_t)blockIdx.y * cols + c], (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    last = __hip_atomic_fetch_add(&tick[blockIdx.x], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
           (int)gridDim.y - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (!last) return;
  const int64_t nrb = gridDim.y;   // the chunk's partial rows, wave w taking rows w, w + 4, ...
  float s = 0.f;
  if (c < cols)
    for (int64_t b = w; b < nrb; b += 4) s += part[b * cols + c];
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && c < cols) out[c] += (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
  if (threadIdx.x == 0) __hip_atomic_store(&tick[blockIdx.x], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// 16 row groups x 64 columns per workgroup: each thread sums nrb / 16 partials (4 in flight), the
// 16 groups combine in LDS in a fixed order
__global__ __launch_bounds__(1024) void colsum_final_kernel(const float* __restrict__ part, int64_t nrb, int64_t cols,
                                                            float* __restrict__ out) {
  __shared__ float red[16][64];
  const int lane = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int64_t c = (int64_t)blockIdx.x * 64 + lane;
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  if (c < cols) {
    int64_t b = grp;
    for (; b + 48 < nrb; b += 64) {
#pragma unroll
      for (int u = 0; u < 4; ++u) a[u] += part[(b + 16 * u) * cols + c];
    }
    for (; b < nrb; b += 16) a[0] += part[b * cols + c];
  }
  red[grp][lane] = (a[0] + a[1]) + (a[2] + a[3]);
  __syncthreads();
  if (grp == 0 && c < cols) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) t += red[q][lane];
    out[c] += t;
  }
}

// blocks: total workgroups to aim for; min_rows: rows per workgroup at least
void colsum_grid(int64_t rows, int64_t cols, int64_t* nrb, int64_t* rb_rows, int64_t blocks = kColsumBlocks,
                 int64_t min_rows = 32) {
  const int64_t cc = (cols + 63) / 64;
  int64_t n = blocks / cc;
  const int64_t by_rows = (rows + min_rows - 1) / min_rows;
  if (n > by_rows) n = by_rows;
  if (n < 1) n = 1;
  *rb_rows = (rows + n - 1) / n;
  *nrb = (rows + *rb_rows - 1) / *rb_rows;
}

}  // namespace

extern "C" int nr_score_fwd(const float* cdd, int64_t ldc, const int64_t* cdd_idx, const float* user,
                            int64_t ldu, int64_t B, int32_t C, int32_t H, int32_t mode, float* logits,
                            hipStream_t stream) {
  if (B < 0 || C < 1 || H < 1 || mode < 0 || mode > 2) return NR_EINVAL(0);
  if (!cdd || !user || !logits) return NR_EINVAL(1);
  if (B == 0) return NR_OK;
  hipLaunchKernelGGL(score_fwd_kernel, dim3((unsigned)B), dim3(256), (size_t)C * sizeof(float), stream, cdd,
                     ldc, cdd_idx, user, ldu, C, H, 1.0f / sqrtf((float)H), mode, logits);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

extern "C" int nr_score_bwd(const float* cdd, int64_t ldc, const float* user, int64_t ldu,
                            const float* logits, const float* dlogits, int64_t B, int32_t C, int32_t H,
                            int32_t mode, float* dcdd, int64_t lddc, float* duser, int64_t lddu,
                            hipStream_t stream) {
  if (B < 0 || C < 1 || H < 1 || mode < 0 || mode > 2) return NR_EINVAL(0);
  if (!cdd || !user || !logits || !dlogits || !dcdd || !duser) return NR_EINVAL(1);
  if (B == 0) return NR_OK;
  hipLaunchKernelGGL(score_bwd_kernel, dim3((unsigned)B), dim3(256), (size_t)C * sizeof(float), stream, cdd,
                     ldc, user, ldu, logits, dlogits, C, H, 1.0f / sqrtf((float)H), mode, dcdd, lddc,
                     duser, lddu);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

extern "C" int nr_score_nll_fwd(const float* cdd, int64_t ldc, const float* user, int64_t ldu,
                                const int64_t* label, int64_t B, int32_t C, int32_t H, float* logits, float* loss,
                                int32_t* work, hipStream_t stream) {
  if (B < 1 || B > 0x7fffffff || C < 1 || C > 16 * 1024 || H < 1) return NR_EINVAL(0);
  if (!cdd || !user || !label || !logits || !loss || !work) return NR_EINVAL(1);
  const int waves = C < 16 ? C : 16;
  hipLaunchKernelGGL(score_nll_fwd_kernel, dim3((unsigned)B), dim3(64 * waves), (size_t)C * sizeof(float), stream,
                     cdd, ldc, user, ldu, label, (int)B, C, H, 1.0f / sqrtf((float)H), logits, loss, work);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

extern "C" int64_t nr_score_nll_workspace(int64_t B) { return 4 + 2 * (B < 0 ? 0 : B); }

extern "C" int nr_score_nll_bwd(const float* cdd, int64_t ldc, const float* user, int64_t ldu,
                                const float* logits, const int64_t* label, const float* dloss,
                                const float* dlogits, int64_t B, int32_t C, int32_t H, float* dcdd, int64_t lddc,
                                float* duser, int64_t lddu, hipStream_t stream) {
  if (B < 0 || C < 1 || H < 1) return NR_EINVAL(0);
  if (!cdd || !user || !logits || !label || !dcdd || !duser) return NR_EINVAL(1);
  if (B == 0) return NR_OK;
  hipLaunchKernelGGL(score_nll_bwd_kernel, dim3((unsigned)B), dim3(256), (size_t)C * sizeof(float), stream, cdd,
                     ldc, user, ldu, logits, label, dloss, dlogits, (int)B, C, H, 1.0f / sqrtf((float)H), dcdd,
                     lddc, duser, lddu);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

extern "C" int nr_adam(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                       float lr, float beta1, float beta2, float eps, float weight_decay, int64_t step,
                       const int64_t* step_dev, float grad_scale, hipStream_t stream) {
  if (n < 0 || (step < 1 && !step_dev)) return NR_EINVAL(0);
  if (!param || !grad || !exp_avg || !exp_avg_sq) return NR_EINVAL(1);
  if ((reinterpret_cast<uintptr_t>(param) | reinterpret_cast<uintptr_t>(grad) |
       reinterpret_cast<uintptr_t>(exp_avg) | reinterpret_cast<uintptr_t>(exp_avg_sq)) & 15)
    return NR_EINVAL(2);
  if (n == 0) return NR_OK;
  // bias corrections in double, as torch computes them in Python floats
  const double bc1 = 1.0 - pow((double)beta1, (double)(step < 1 ? 1 : step));
  const double bc2 = 1.0 - pow((double)beta2, (double)(step < 1 ? 1 : step));
  int64_t blocks = (n / 4 + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, param, grad, exp_avg,
                     exp_avg_sq, n, (float)((double)lr / bc1), beta1, beta2, eps, (float)sqrt(bc2), weight_decay, grad_scale,
                     step_dev, lr);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

extern "C" int nr_embedding_fwd(const float* table, int64_t V, int64_t E, const int64_t* idx, int64_t n,
                                float* out, hipStream_t stream) {
  if (V < 1 || E < 4 || (E & 3) || n < 0) return NR_EINVAL(0);
  if (!table || !idx || !out) return NR_EINVAL(1);
  if (n == 0) return NR_OK;
  hipLaunchKernelGGL(embedding_fwd_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, stream, table, E, idx,
                     n, out);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

extern "C" int nr_embedding_bwd(const float* dout, int64_t V, int64_t E, const int64_t* idx, int64_t n,
                                int64_t padding_idx, float* dtable, hipStream_t stream) {
  if (V < 1 || E < 1 || n < 0) return NR_EINVAL(0);
  if (!dout || !idx || !dtable) return NR_EINVAL(1);
  if (n == 0) return NR_OK;
  hipLaunchKernelGGL(embedding_bwd_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, stream, dout, E, idx,
                     n, padding_idx, dtable);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

extern "C" int nr_rows_add_ordered(const float* dout, int64_t ldo, int64_t V, int64_t E, const int64_t* idx, int64_t n,
                                   int64_t padding_idx, float* dtable, int64_t ldt, hipStream_t stream) {
  if (V < 1 || E < 1 || n < 0 || n > (1 << 20) || ldo < E || ldt < E) return NR_EINVAL(0);
  if (!dout || !idx || !dtable) return NR_EINVAL(1);
  if (n == 0) return NR_OK;
  hipLaunchKernelGGL(rows_add_ordered_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, stream, dout, ldo, V, E,
                     idx, n, padding_idx, dtable, ldt);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

extern "C" int nr_xsoftmax_fwd(const float* x, const void* mask, int32_t mask_dtype, int64_t rows, int64_t cols,
                               float* out, hipStream_t stream) {
  if (rows < 0 || cols < 0 || mask_dtype < NR_MASK_U8 || mask_dtype > NR_MASK_F32) return NR_EINVAL(0);
  if (!x || !mask || !out) return NR_EINVAL(1);
  if (rows == 0 || cols == 0) return NR_OK;
  hipLaunchKernelGGL(xsoftmax_fwd_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, stream, x, mask, mask_dtype,
                     rows, cols, out);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

extern "C" int nr_xsoftmax_bwd(const float* y, const float* dy, int64_t rows, int64_t cols, float* dx,
                               hipStream_t stream) {
  if (rows < 0 || cols < 0) return NR_EINVAL(0);
  if (!y || !dy || !dx) return NR_EINVAL(1);
  if (rows == 0 || cols == 0) return NR_OK;
  hipLaunchKernelGGL(xsoftmax_bwd_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, stream, y, dy, rows, cols,
                     dx);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

extern "C" int nr_gather_rows_f32(const float* src, int64_t lds, int64_t V, const int64_t* idx, int64_t n,
                                  int64_t cols, float* dst, int64_t ldd, hipStream_t stream) {
  if (n < 0 || cols < 0 || V < 1 || lds < cols || ldd < cols) return NR_EINVAL(0);
  if (!src || !idx || !dst) return NR_EINVAL(1);
  if (n == 0 || cols == 0) return NR_OK;
  const int vec4 = ((cols | lds | ldd) & 3) == 0 && ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0;
  hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, stream, src, lds, idx, n, cols, dst,
                     ldd, vec4);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

extern "C" int nr_transpose_f32(const float* src, int64_t lds, int64_t rows, int64_t cols, float* dst, int64_t ldd,
                                hipStream_t stream) {
  if (rows < 0 || cols < 0 || lds < cols || ldd < rows || rows > (int64_t)65535 * 64 || cols > ((int64_t)1 << 31))
    return NR_EINVAL(0);
  if (!src || !dst) return NR_EINVAL(1);
  if (rows == 0 || cols == 0) return NR_OK;
  hipLaunchKernelGGL(transpose_kernel, dim3((unsigned)((cols + 63) / 64), (unsigned)((rows + 63) / 64)), dim3(256), 0,
                     stream, src, lds, rows, cols, dst, ldd);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

extern "C" int64_t nr_colsum_workspace(int64_t rows, int64_t cols) {
  if (rows <= 0 || cols <= 0) return 0;
  int64_t nrb, rb_rows;
  colsum_grid(rows, cols, &nrb, &rb_rows);
  return nrb * cols * (int64_t)sizeof(float);
}

extern "C" int nr_colsum(const float* x, int64_t ldx, int64_t rows, int64_t cols, float* out, float* work,
                         hipStream_t stream) {
  if (rows < 0 || cols < 0 || ldx < cols) return NR_EINVAL(0);
  if (!x || !out || (rows > 0 && cols > 0 && !work)) return NR_EINVAL(1);
  if (rows == 0 || cols == 0) return NR_OK;
  int64_t nrb, rb_rows;
  colsum_grid(rows, cols, &nrb, &rb_rows);
  hipLaunchKernelGGL(colsum_part_kernel, dim3((unsigned)((cols + 63) / 64), (unsigned)nrb), dim3(256), 0, stream, x,
                     ldx, rows, cols, rb_rows, work, nullptr, nullptr);
  hipLaunchKernelGGL(colsum_final_kernel, dim3((unsigned)((cols + 63) / 64)), dim3(1024), 0, stream, work, nrb, cols,
                     out);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

extern "C" int nr_colsum_ws(const float* x, int64_t ldx, int64_t rows, int64_t cols, float* out, float* work,
                            int32_t* tick, hipStream_t stream) {
  if (rows < 0 || cols < 0 || ldx < cols) return NR_EINVAL(0);
  if (!x || !out || (rows > 0 && cols > 0 && (!work || !tick))) return NR_EINVAL(1);
  if (rows == 0 || cols == 0) return NR_OK;
  // one round of workgroups (fewer, longer partials: the last arriver of a chunk reads them all)
  int64_t nrb, rb_rows;
  colsum_grid(rows, cols, &nrb, &rb_rows, 512, 128);
  hipLaunchKernelGGL(colsum_part_kernel, dim3((unsigned)((cols + 63) / 64), (unsigned)nrb), dim3(256), 0, stream, x,
                     ldx, rows, cols, rb_rows, work, tick, out);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

namespace {
int adam_multi_launch(AdamMulti& a, int64_t blocks, hipStream_t stream) {
  if (a.count == 0) return NR_OK;
  // only empty tensors (ticket launches): one block with no elements advances their step counts
  if (blocks == 0) blocks = 1;
  a.blk_off[a.count] = (int32_t)blocks;
  hipLaunchKernelGGL(adam_multi_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, a);
  NR_LAUNCH_CHECK();
  return NR_OK;
}
}  // namespace

namespace {
int adam_multi_impl(const nr_adam_tensor* tensors, int32_t count, float beta1, float beta2, float eps,
                    float weight_decay, float grad_scale, int32_t* ticket, hipStream_t stream) {
  if (count < 0 || (count > 0 && !tensors)) return NR_EINVAL(0);
  for (int32_t t = 0; t < count; ++t) {   // validate everything before the first launch
    const nr_adam_tensor& d = tensors[t];
    if (d.n < 0 || (d.step < 1 && !d.step_dev)) return NR_EINVAL(1);
    if (d.n > 0 && (!d.param || !d.grad || !d.exp_avg || !d.exp_avg_sq)) return NR_EINVAL(2);
    if ((d.n + kAdamChunk - 1) / kAdamChunk > 0x3fffffff) return NR_EINVAL(3);
    if (d.row_touched && d.row_len < 1) return NR_EINVAL(5);
  }
  AdamMulti a;
  a.b1 = beta1; a.b2 = beta2; a.eps = eps; a.wd = weight_decay; a.gscale = grad_scale;
  a.count = 0;
  a.ticket = ticket;
  int64_t blocks = 0;
  for (int32_t t = 0; t < count; ++t) {
    const nr_adam_tensor& d = tensors[t];
    // an empty tensor has no work; with a ticket it still takes an entry (no blocks) so that the
    // launch advances its device step count, as torch's capturable Adam does for every parameter
    // with a gradient
    if (d.n == 0 && !(ticket && d.step_dev)) continue;
    const int64_t nb = (d.n + kAdamChunk - 1) / kAdamChunk;
    if (a.count == kAdamMulti || blocks + nb > 0x7fffffff) {
      const int rc = adam_multi_launch(a, blocks, stream);
      if (rc) return rc;
      a.count = 0;
      blocks = 0;
    }
    AdamEntry& e = a.e[a.count];
    e.p = d.param; e.g = d.grad; e.m = d.exp_avg; e.v = d.exp_avg_sq; e.n = d.n;
    e.step_dev = const_cast<int64_t*>(d.step_dev); e.lr_dev = d.lr_dev; e.lr = d.lr;
    e.rt = d.row_touched; e.rlen = d.row_touched ? d.row_len : 1;
    const double st = (double)(d.step < 1 ? 1 : d.step);   // bias corrections in double, as torch's Python floats
    e.step = (int64_t)st;
    e.step_size = (float)((double)d.lr / (1.0 - pow((double)beta1, st)));
    e.bc2_sqrt = (float)sqrt(1.0 - pow((double)beta2, st));
    a.blk_off[a.count] = (int32_t)blocks;
    blocks += nb;
    ++a.count;
  }
  return adam_multi_launch(a, blocks, stream);
}
}  // namespace

extern "C" int nr_adam_multi(const nr_adam_tensor* tensors, int32_t count, float beta1, float beta2, float eps,
                             float weight_decay, float grad_scale, hipStream_t stream) {
  return adam_multi_impl(tensors, count, beta1, beta2, eps, weight_decay, grad_scale, nullptr, stream);
}

extern "C" int nr_adam_multi_step(const nr_adam_tensor* tensors, int32_t count, float beta1, float beta2, float eps,
                                  float weight_decay, float grad_scale, int32_t* ticket, hipStream_t stream) {
  if (!ticket) return NR_EINVAL(4);
  return adam_multi_impl(tensors, count, beta1, beta2, eps, weight_decay, grad_scale, ticket, stream);
}
