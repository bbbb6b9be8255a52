// Learned-query attention pooling WITHOUT LayerNorm / dropout, one wave per sequence:
//   s_l = scale * q · K_l   (K = a separate key matrix, or X itself: tied)
//   p   = XSoftmax(s, mask) (masked -> exactly 0; a fully masked sequence -> all zeros)
//   out = Σ_l p_l X_l
// Call sites: CNN_Encoder's word pooling (CNN.py:46, key = tanh(W c + b)) and Attention_Pooling
// (Pooling.py:22-24, tied key).  nr_attn_pool_* (attn_pool.hip) keeps the LN / dropout forms.
//
// A wave owns a whole sequence: lane j holds features 4j .. 4j + 3 (D <= 256; any D: the lane that
// straddles D reads and writes its valid features only), rows stream through
// as coalesced float4 row segments, eight in flight; the per-row dot products are wave reductions
// whose results every lane keeps, so the softmax and its backward need no LDS and no barrier.  The
// workgroup-per-sequence form staged the rows in LDS and ran its dq / dK loop one feature per thread
// serially over the rows (latency-bound: 69 us per CNN step for 52.8 k rows).  dq is summed per
// workgroup over its sequences and added with one atomic per feature per workgroup.
#include "common.h"
#include "../../include/newsrec_hip.h"

namespace {

constexpr int SP_WAVES = 4;

struct SeqPoolArgs {
  const float* x; int64_t ldx;
  const float* key; int64_t ldk;   // NULL: tied
  const float* q;
  const void* mask; int mask_dt;
  int64_t nseq; int L; int D; int qn; float scale;   // qn: valid length of q and of a dout row (<= D)
  float* out; int64_t ldo;
  float* probs;
  // backward
  const float* dout; int64_t lddo;
  const float* dz; int64_t lddz;
  float* dx; int64_t lddx;
  float* dk; int64_t lddk; int key_tanh;
  float* dq;
};

// features 4j .. 4j+3 of a 16-B aligned row (ld % 4 == 0, ld >= round4(D)): always one float4 load
// at a column clamped into the row, features >= D zeroed by selects -- branch-free, so the compiler
// keeps every row load of a batch in flight (a branch around a load makes it wait at the join)
__device__ __forceinline__ float4 ld4(const float* row, int j, int D) {
  const int last = ((D + 3) & ~3) - 4;
  const int c = 4 * j < last ? 4 * j : last;
  const float4 v = *reinterpret_cast<const float4*>(row + c);
  return make_float4(4 * j < D ? v.x : 0.f, 4 * j + 1 < D ? v.y : 0.f, 4 * j + 2 < D ? v.z : 0.f,
                     4 * j + 3 < D ? v.w : 0.f);
}

__device__ __forceinline__ void st4(float* row, int j, int D, float4 v) {
  if (4 * j + 3 < D) {
    *reinterpret_cast<float4*>(row + 4 * j) = v;
    return;
  }
  if (4 * j < D) row[4 * j] = v.x;
  if (4 * j + 1 < D) row[4 * j + 1] = v.y;
  if (4 * j + 2 < D) row[4 * j + 2] = v.z;
}

// features 4j .. 4j+3 of an unaligned vector of n valid floats (q, a dout row): scalar loads at
// clamped indices, zeroed past n by selects (branch-free)
__device__ __forceinline__ float4 ldv(const float* v, int j, int n) {
  float e[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int i = 4 * j + u;
    const float x = v[i < n ? i : n - 1];
    e[u] = i < n ? x : 0.f;
  }
  return make_float4(e[0], e[1], e[2], e[3]);
}

__device__ __forceinline__ float dot4(float4 a, float4 b) { return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w; }

// s[l] = scale * q · K_l for l < L (every lane holds every score)
template <int SP_MAXL>
__device__ __forceinline__ void scores(const SeqPoolArgs& g, int64_t seq, int lane, float4 qv, float (&s)[SP_MAXL]) {
  const float* kb = g.key ? g.key + seq * g.L * g.ldk : g.x + seq * g.L * g.ldx;
  const int64_t ld = g.key ? g.ldk : g.ldx;
  // every slot computed (rows past L clamped, masked later): fully unrolled, no dynamic indexing
#pragma unroll
  for (int l0 = 0; l0 < SP_MAXL; l0 += 8) {
    float part[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int l = l0 + u < g.L ? l0 + u : g.L - 1;
      part[u] = dot4(qv, ld4(kb + l * ld, lane, g.D));
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) s[l0 + u] = nr_wave_sum(part[u]) * g.scale;
  }
}

// softmax with the XSoftmax mask semantics; p[l] for l < L (0 for masked / l >= L)
template <int SP_MAXL>
__device__ __forceinline__ void softmax(const SeqPoolArgs& g, int64_t seq, float (&s)[SP_MAXL]) {
  const int lane = threadIdx.x & 63;
  const uint64_t bits = __ballot(lane < g.L && nr_mask_at(g.mask, g.mask_dt, seq * g.L + lane));
  float mx = -INFINITY;
#pragma unroll
  for (int l = 0; l < SP_MAXL; ++l)
    if (l < g.L && ((bits >> l) & 1ull)) mx = fmaxf(mx, s[l]);
  float sum = 0.f;
#pragma unroll
  for (int l = 0; l < SP_MAXL; ++l) {
    const float e = (l < g.L && ((bits >> l) & 1ull)) ? __expf(s[l] - mx) : 0.f;
    s[l] = e;
    sum += e;
  }
  const float inv = sum > 0.f ? 1.f / sum : 0.f;
#pragma unroll
  for (int l = 0; l < SP_MAXL; ++l) s[l] *= inv;
}

template <int SP_MAXL>
__global__ __launch_bounds__(64 * SP_WAVES) void seq_pool_fwd_kernel(SeqPoolArgs g) {
  const int lane = threadIdx.x & 63;
  const int64_t seq = (int64_t)blockIdx.x * SP_WAVES + (threadIdx.x >> 6);
  if (seq >= g.nseq) return;
  const float4 qv = ldv(g.q, lane, g.qn);
  float s[SP_MAXL];
  scores<SP_MAXL>(g, seq, lane, qv, s);
  softmax<SP_MAXL>(g, seq, s);
  if (lane < g.L) {
    float pl = 0.f;
#pragma unroll
    for (int l = 0; l < SP_MAXL; ++l) pl = l == lane ? s[l] : pl;
    g.probs[seq * g.L + lane] = pl;
  }
  const float* xb = g.x + seq * g.L * g.ldx;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int l = 0; l < SP_MAXL; ++l) {   // s[l] = 0 past L
    const float4 v = ld4(xb + (l < g.L ? l : g.L - 1) * g.ldx, lane, g.D);
    acc.x = fmaf(s[l], v.x, acc.x); acc.y = fmaf(s[l], v.y, acc.y);
    acc.z = fmaf(s[l], v.z, acc.z); acc.w = fmaf(s[l], v.w, acc.w);
  }
  st4(g.out + seq * g.ldo, lane, g.D, acc);
}

// grid-stride over the sequences (one per wave per round) so that dq is reduced over many
// sequences per workgroup before its one atomic per feature
template <int SP_MAXL>
__global__ __launch_bounds__(64 * SP_WAVES) void seq_pool_bwd_kernel(SeqPoolArgs g) {
  __shared__ float4 red[SP_WAVES][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float4 qv = ldv(g.q, lane, g.qn);
  float4 dqa = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int64_t seq = (int64_t)blockIdx.x * SP_WAVES + w; seq < g.nseq; seq += (int64_t)gridDim.x * SP_WAVES) {
    const float* xb = g.x + seq * g.L * g.ldx;
    const float* kb = g.key ? g.key + seq * g.L * g.ldk : xb;
    const int64_t ldk = g.key ? g.ldk : g.ldx;
    // per-row scalars live one per lane (lane l: p_l, dp_l, ds_l) and are broadcast with v_readlane
    // where a row is used: two VGPRs instead of two 32-entry arrays replicated in every lane
    const float pv = lane < g.L ? g.probs[seq * g.L + lane] : 0.f;
    const float4 dov = ldv(g.dout + seq * g.lddo, lane, g.qn);
    // dp_l = dout · X_l
    float dpv = 0.f;
#pragma unroll
    for (int l0 = 0; l0 < SP_MAXL; l0 += 8) {
      float part[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int l = l0 + u < g.L ? l0 + u : g.L - 1;
        part[u] = dot4(dov, ld4(xb + l * g.ldx, lane, g.D));
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float t = nr_wave_sum(part[u]);
        dpv = lane == l0 + u ? t : dpv;
      }
    }
    const float r = nr_wave_sum(lane < g.L ? pv * dpv : 0.f);
    const float dsv = pv * (dpv - r) * g.scale;
    // ds_l = p_l (dp_l - r) scale;  dq += ds_l K_l;  dK_l = ds_l q (tanh');  dX_l = p_l dout (+ ds_l q tied) (+ dz)
    // eight rows at a time: their key / dz loads go out together before any store of the batch
#pragma unroll
    for (int l0 = 0; l0 < SP_MAXL; l0 += 8) {
      if (l0 >= g.L) break;   // wave-uniform; the batches below are fully unrolled
      float4 kv[8], zv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int l = l0 + u < g.L ? l0 + u : g.L - 1;
        kv[u] = ld4(kb + l * ldk, lane, g.D);
        zv[u] = g.dz ? ld4(g.dz + (seq * g.L + l) * g.lddz, lane, g.D) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int l = l0 + u;
        if (l >= g.L) break;
        const float pl = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pv), l));
        const float ds = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dsv), l));
        dqa.x = fmaf(ds, kv[u].x, dqa.x); dqa.y = fmaf(ds, kv[u].y, dqa.y);
        dqa.z = fmaf(ds, kv[u].z, dqa.z); dqa.w = fmaf(ds, kv[u].w, dqa.w);
        const int64_t row = seq * g.L + l;
        float4 dxv = make_float4(pl * dov.x + zv[u].x, pl * dov.y + zv[u].y, pl * dov.z + zv[u].z, pl * dov.w + zv[u].w);
        if (g.key) {
          float4 dkv = make_float4(ds * qv.x, ds * qv.y, ds * qv.z, ds * qv.w);
          if (g.key_tanh) {
            dkv.x *= 1.f - kv[u].x * kv[u].x; dkv.y *= 1.f - kv[u].y * kv[u].y;
            dkv.z *= 1.f - kv[u].z * kv[u].z; dkv.w *= 1.f - kv[u].w * kv[u].w;
          }
          st4(g.dk + row * g.lddk, lane, g.D, dkv);
        } else {
          dxv.x = fmaf(ds, qv.x, dxv.x); dxv.y = fmaf(ds, qv.y, dxv.y);
          dxv.z = fmaf(ds, qv.z, dxv.z); dxv.w = fmaf(ds, qv.w, dxv.w);
        }
        st4(g.dx + row * g.lddx, lane, g.D, dxv);
      }
    }
  }
  red[w][lane] = dqa;
  __syncthreads();
  if (w == 0 && 4 * lane < g.qn) {
    float4 t = red[0][lane];
#pragma unroll
    for (int ww = 1; ww < SP_WAVES; ++ww) {
      const float4 v = red[ww][lane];
      t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
    }
    const float e[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (4 * lane + u < g.qn) atomicAdd(&g.dq[4 * lane + u], e[u]);
  }
}

// ---- workgroup per sequence (L <= 64, D <= 64 * 4 * NF; NF = 1, 2, 4: D <= 1024)
constexpr int WG_WAVES = 8;
constexpr int WG_RPW = 64 / WG_WAVES;   // rows per wave

template <int NF>
__global__ __launch_bounds__(64 * WG_WAVES) void seq_pool_wg_fwd_kernel(SeqPoolArgs g) {
  __shared__ float sc[64];
  __shared__ float4 red[WG_WAVES][64 * NF];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t seq = blockIdx.x;
  const float* xb = g.x + seq * g.L * g.ldx;
  const float* kb = g.key ? g.key + seq * g.L * g.ldk : xb;
  const int64_t ldk = g.key ? g.ldk : g.ldx;
  float4 qv[NF], kv[WG_RPW][NF];
#pragma unroll
  for (int f = 0; f < NF; ++f) qv[f] = ldv(g.q, lane + 64 * f, g.qn);
#pragma unroll
  for (int k = 0; k < WG_RPW; ++k) {
    const int l = w + WG_WAVES * k, lc = l < g.L ? l : g.L - 1;
#pragma unroll
    for (int f = 0; f < NF; ++f) kv[k][f] = ld4(kb + lc * ldk, lane + 64 * f, g.D);
  }
#pragma unroll
  for (int k = 0; k < WG_RPW; ++k) {
    float d = 0.f;
#pragma unroll
    for (int f = 0; f < NF; ++f) d += dot4(qv[f], kv[k][f]);
    d = nr_wave_sum(d);
    const int l = w + WG_WAVES * k;
    if (lane == 0 && l < g.L) sc[l] = d * g.scale;
  }
  __syncthreads();
  // softmax (every wave, lane l = row l) with XSoftmax's mask semantics
  const bool keep = lane < g.L && nr_mask_at(g.mask, g.mask_dt, seq * g.L + lane);
  const float v = keep ? sc[lane] : -INFINITY;
  const float mx = nr_wave_max(v);
  const float e = keep ? __expf(v - mx) : 0.f;
  const float sum = nr_wave_sum(e);
  const float p = sum > 0.f ? e / sum : 0.f;
  if (w == 0 && lane < g.L) g.probs[seq * g.L + lane] = p;
  float4 acc[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f) acc[f] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int k = 0; k < WG_RPW; ++k) {
    const int l = w + WG_WAVES * k, lc = l < g.L ? l : g.L - 1;
    const float pl = __shfl(p, l & 63, 64);   // 0 for l >= L (lane l has p = 0 there)
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      const float4 xv = g.key ? ld4(xb + lc * g.ldx, lane + 64 * f, g.D) : kv[k][f];
      acc[f].x = fmaf(pl, xv.x, acc[f].x); acc[f].y = fmaf(pl, xv.y, acc[f].y);
      acc[f].z = fmaf(pl, xv.z, acc[f].z); acc[f].w = fmaf(pl, xv.w, acc[f].w);
    }
  }
#pragma unroll
  for (int f = 0; f < NF; ++f) red[w][lane + 64 * f] = acc[f];
  __syncthreads();
  for (int j = threadIdx.x; j < 64 * NF && 4 * j < g.D; j += 64 * WG_WAVES) {
    float4 t = red[0][j];
#pragma unroll
    for (int ww = 1; ww < WG_WAVES; ++ww) {
      const float4 u = red[ww][j];
      t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
    }
    st4(g.out + seq * g.ldo, j, g.D, t);
  }
}

template <int NF>
__global__ __launch_bounds__(64 * WG_WAVES) void seq_pool_wg_bwd_kernel(SeqPoolArgs g) {
  __shared__ float dps[64];
  __shared__ float4 red[WG_WAVES][64 * NF];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t seq = blockIdx.x;
  const float* xb = g.x + seq * g.L * g.ldx;
  const float* kb = g.key ? g.key + seq * g.L * g.ldk : xb;
  const int64_t ldk = g.key ? g.ldk : g.ldx;
  float4 qv[NF], dov[NF], xv[WG_RPW][NF];
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    qv[f] = ldv(g.q, lane + 64 * f, g.qn);
    dov[f] = ldv(g.dout + seq * g.lddo, lane + 64 * f, g.qn);
  }
  const float pme = lane < g.L ? g.probs[seq * g.L + lane] : 0.f;   // lane l: p_l
#pragma unroll
  for (int k = 0; k < WG_RPW; ++k) {
    const int l = w + WG_WAVES * k, lc = l < g.L ? l : g.L - 1;
#pragma unroll
    for (int f = 0; f < NF; ++f) xv[k][f] = ld4(xb + lc * g.ldx, lane + 64 * f, g.D);
  }
  // dp_l = dout · X_l
#pragma unroll
  for (int k = 0; k < WG_RPW; ++k) {
    float d = 0.f;
#pragma unroll
    for (int f = 0; f < NF; ++f) d += dot4(dov[f], xv[k][f]);
    d = nr_wave_sum(d);
    const int l = w + WG_WAVES * k;
    if (lane == 0 && l < g.L) dps[l] = d;
  }
  __syncthreads();
  const float dpme = lane < g.L ? dps[lane] : 0.f;
  const float r = nr_wave_sum(pme * dpme);
  float4 dqa[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f) dqa[f] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int k = 0; k < WG_RPW; ++k) {
    const int l = w + WG_WAVES * k;
    const float pl = __shfl(pme, l & 63, 64), dpl = __shfl(dpme, l & 63, 64);
    if (l >= g.L) continue;   // wave-uniform
    const float ds = pl * (dpl - r) * g.scale;
    const int64_t row = seq * g.L + l;
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      const int j = lane + 64 * f;
      const float4 kv = g.key ? ld4(kb + l * ldk, j, g.D) : xv[k][f];
      dqa[f].x = fmaf(ds, kv.x, dqa[f].x); dqa[f].y = fmaf(ds, kv.y, dqa[f].y);
      dqa[f].z = fmaf(ds, kv.z, dqa[f].z); dqa[f].w = fmaf(ds, kv.w, dqa[f].w);
      const float4 zv = g.dz ? ld4(g.dz + row * g.lddz, j, g.D) : make_float4(0.f, 0.f, 0.f, 0.f);
      float4 dxv = make_float4(fmaf(pl, dov[f].x, zv.x), fmaf(pl, dov[f].y, zv.y), fmaf(pl, dov[f].z, zv.z),
                               fmaf(pl, dov[f].w, zv.w));
      if (g.key) {
        float4 dkv = make_float4(ds * qv[f].x, ds * qv[f].y, ds * qv[f].z, ds * qv[f].w);
        if (g.key_tanh) {
          dkv.x *= 1.f - kv.x * kv.x; dkv.y *= 1.f - kv.y * kv.y;
          dkv.z *= 1.f - kv.z * kv.z; dkv.w *= 1.f - kv.w * kv.w;
        }
        if (4 * j < g.D) st4(g.dk + row * g.lddk, j, g.D, dkv);
      } else {
        dxv.x = fmaf(ds, qv[f].x, dxv.x); dxv.y = fmaf(ds, qv[f].y, dxv.y);
        dxv.z = fmaf(ds, qv[f].z, dxv.z); dxv.w = fmaf(ds, qv[f].w, dxv.w);
      }
      if (4 * j < g.D) st4(g.dx + row * g.lddx, j, g.D, dxv);
    }
  }
#pragma unroll
  for (int f = 0; f < NF; ++f) red[w][lane + 64 * f] = dqa[f];
  __syncthreads();
  for (int j = threadIdx.x; j < 64 * NF && 4 * j < g.qn; j += 64 * WG_WAVES) {
    float4 t = red[0][j];
#pragma unroll
    for (int ww = 1; ww < WG_WAVES; ++ww) {
      const float4 u = red[ww][j];
      t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
    }
    const float e4[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (4 * j + u < g.qn) atomicAdd(&g.dq[4 * j + u], e4[u]);
  }
}

// the workgroup form for long features (D > 256) or few sequences (< 4 waves per CU of the
// wave-per-sequence form)
bool use_wg(int64_t nseq, int D) { return D > 256 || nseq < 1024; }

bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

int64_t r4(int D) { return (D + 3) & ~3; }

bool shape_ok(int L, int D, int qn, int64_t ldx, int64_t ldk, const void* x, const void* key) {
  return L >= 1 && L <= 64 && D >= 1 && D <= 1024 && qn >= 1 && qn <= D && ldx >= r4(D) && (ldx & 3) == 0 && al16(x) &&
         (!key || ((ldk & 3) == 0 && ldk >= r4(D) && al16(key)));
}

}  // namespace

extern "C" int nr_seq_pool_fwd(const float* x, int64_t ldx, const float* key, int64_t ldk, const float* q,
                               int32_t qn, const void* mask, int32_t mask_dtype, int64_t nseq, int32_t L, int32_t D,
                               float scale, float* out, int64_t ldo, float* probs, hipStream_t stream) {
  if (!shape_ok(L, D, qn, ldx, ldk, x, key) || (ldo & 3) || ldo < D || nseq < 0) return NR_EINVAL(0);
  if (!x || !q || !mask || !out || !probs) return NR_EINVAL(1);
  if (!al16(out)) return NR_EINVAL(2);
  if (nseq == 0) return NR_OK;
  SeqPoolArgs g{};
  g.x = x; g.ldx = ldx; g.key = key; g.ldk = ldk; g.q = q; g.mask = mask; g.mask_dt = mask_dtype;
  g.nseq = nseq; g.L = L; g.D = D; g.qn = qn; g.scale = scale; g.out = out; g.ldo = ldo; g.probs = probs;
  if (use_wg(nseq, D)) {
    if (D <= 256)
      hipLaunchKernelGGL(seq_pool_wg_fwd_kernel<1>, dim3((unsigned)nseq), dim3(64 * WG_WAVES), 0, stream, g);
    else if (D <= 512)
      hipLaunchKernelGGL(seq_pool_wg_fwd_kernel<2>, dim3((unsigned)nseq), dim3(64 * WG_WAVES), 0, stream, g);
    else   // BERT-width history vectors (the 768-wide MHA user encoder)
      hipLaunchKernelGGL(seq_pool_wg_fwd_kernel<4>, dim3((unsigned)nseq), dim3(64 * WG_WAVES), 0, stream, g);
    NR_LAUNCH_CHECK();
    return NR_OK;
  }
  const dim3 grid((unsigned)((nseq + SP_WAVES - 1) / SP_WAVES));
  if (L <= 32)
    hipLaunchKernelGGL(seq_pool_fwd_kernel<32>, grid, dim3(64 * SP_WAVES), 0, stream, g);
  else
    hipLaunchKernelGGL(seq_pool_fwd_kernel<64>, grid, dim3(64 * SP_WAVES), 0, stream, g);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

extern "C" int nr_seq_pool_bwd(const float* x, int64_t ldx, const float* key, int64_t ldk, const float* q,
                               int32_t qn, const void* mask, int32_t mask_dtype, int64_t nseq, int32_t L, int32_t D,
                               float scale, const float* probs, const float* dout, int64_t lddo, const float* dz,
                               int64_t lddz, float* dx, int64_t lddx, float* dk, int64_t lddk, int32_t key_tanh,
                               float* dq, hipStream_t stream) {
  if (!shape_ok(L, D, qn, ldx, ldk, x, key) || lddo < qn || (lddx & 3) || lddx < D ||
      (dz && ((lddz & 3) || lddz < r4(D))) || (key && ((lddk & 3) || lddk < D)) || nseq < 0)
    return NR_EINVAL(0);
  if (!x || !q || !mask || !probs || !dout || !dx || !dq || (key && !dk)) return NR_EINVAL(1);
  if (!al16(dx) || (dz && !al16(dz)) || (dk && !al16(dk))) return NR_EINVAL(2);
  if (nseq == 0) return NR_OK;
  SeqPoolArgs g{};
  g.x = x; g.ldx = ldx; g.key = key; g.ldk = ldk; g.q = q; g.mask = mask; g.mask_dt = mask_dtype;
  g.nseq = nseq; g.L = L; g.D = D; g.qn = qn; g.scale = scale; g.probs = const_cast<float*>(probs);
  g.dout = dout; g.lddo = lddo; g.dz = dz; g.lddz = lddz; g.dx = dx; g.lddx = lddx; g.dk = dk; g.lddk = lddk;
  g.key_tanh = key_tanh; g.dq = dq;
  if (use_wg(nseq, D)) {
    if (D <= 256)
      hipLaunchKernelGGL(seq_pool_wg_bwd_kernel<1>, dim3((unsigned)nseq), dim3(64 * WG_WAVES), 0, stream, g);
    else if (D <= 512)
      hipLaunchKernelGGL(seq_pool_wg_bwd_kernel<2>, dim3((unsigned)nseq), dim3(64 * WG_WAVES), 0, stream, g);
    else
      hipLaunchKernelGGL(seq_pool_wg_bwd_kernel<4>, dim3((unsigned)nseq), dim3(64 * WG_WAVES), 0, stream, g);
    NR_LAUNCH_CHECK();
    return NR_OK;
  }
  int64_t blocks = (nseq + SP_WAVES - 1) / SP_WAVES;
  if (blocks > 1024) blocks = 1024;   // dq: one atomic per feature per workgroup
  if (L <= 32)
    hipLaunchKernelGGL(seq_pool_bwd_kernel<32>, dim3((unsigned)blocks), dim3(64 * SP_WAVES), 0, stream, g);
  else
    hipLaunchKernelGGL(seq_pool_bwd_kernel<64>, dim3((unsigned)blocks), dim3(64 * SP_WAVES), 0, stream, g);
  NR_LAUNCH_CHECK();
  return NR_OK;
}
