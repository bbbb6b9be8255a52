// BERT tower kernels (transformers BertModel as XFormer / PLM call it: models/XFormer.py:68,94,
// models/PLM.py:102,121).  The dense layers run on nr_gemm_f32 (QKV, attention output,
// intermediate with a fused GELU epilogue, output, pooler with a tanh epilogue); this file holds
// everything between the GEMMs:
//
//   nr_bert_embed_fwd / _bwd   word + position + token-type rows -> LayerNorm -> dropout
//   nr_bert_add_ln_fwd / _bwd  LayerNorm(dropout(dense) + residual)     (BertSelfOutput/BertOutput)
//   nr_bert_attn_fwd           softmax(Q Kᵀ / 8 + additive key mask) -> dropout -> · V per
//                              (sequence, head), online softmax, any L; products on the f32
//                              MFMA or the bf16 MFMA (bf16x6 / bf16, per the caller's precision)
//   nr_bert_attn_bwd           dQ, dK, dV from the saved per-query (max, 1/sum)
//   nr_tanh_bwd                pooler tanh backward
//
// Attention tiling (head dim 64).  A wave owns 32 rows (queries in the forward / dQ pass, keys
// in the dK/dV pass); the workgroup's waves share LDS-staged 32-row tiles of the other side.
// Scores are formed TRANSPOSED where the softmax statistics are per query: Sᵀ = K Qᵀ puts the
// query on the lane (column of the 32x32 C tile), so a query's max / sum / rescale is lane-local
// up to one swap of the two lane halves, and the accumulator tile is directly the B operand of
// the next MFMA (Oᵀ = Vᵀ Pᵀ): k-step s of that product takes key kr(s, h) = 8(s>>2) + 4h + (s&3),
// which is the row accumulator register s of lane half h holds.  The contraction over the 64
// head dims uses dim 32h + s in k-step s (the order is free), so every operand fragment is 32
// consecutive floats of one row.
#include "common.h"
#include "mfma_planes.h"
#include "../../include/newsrec_hip.h"

namespace {

constexpr float kNegMax = -3.4028234663852886e38f;   // torch.finfo(float32).min
constexpr int kHD = 64;                               // head dim
constexpr int kLS = 68;                               // LDS row stride (floats)

__device__ __forceinline__ float xhalf_sum(float v) {   // v(lane) + v(lane ^ 32)
  const unsigned x = __builtin_bit_cast(unsigned, v);
  auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  return __builtin_bit_cast(float, (unsigned)r[0]) + __builtin_bit_cast(float, (unsigned)r[1]);
}
__device__ __forceinline__ float xhalf_max(float v) {
  const unsigned x = __builtin_bit_cast(unsigned, v);
  auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  return fmaxf(__builtin_bit_cast(float, (unsigned)r[0]), __builtin_bit_cast(float, (unsigned)r[1]));
}

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }

// ------------------------------------------------------------------------------------ LayerNorm rows
// One wave per row of H floats (H % 4 == 0, H <= 256 * NV); lane owns float4 chunks lane + 64 j.

struct LnArgs {
  // inputs of the LayerNorm's argument s
  const float* word; int64_t V; const float* pos; const float* type0; const int64_t* ids; int L;   // embed
  const float* x; int64_t ldx; const float* res; int64_t ldr;                                      // add
  int64_t T; int H;
  const float* gamma; const float* beta; float eps;
  float p; float pscale; uint32_t thresh; uint32_t key; const uint64_t* rng; uint64_t offset;
  float* out; int64_t ldo; float* stats;   // stats written by the forward, read by the backward
  // backward
  const float* dout; int64_t ldd;
  float* ds; int64_t ldds;     // embed: dL/ds ; add: dL/dres
  float* dx; int64_t lddx;     // add: dL/d(dense)
  float* dgamma; float* dbeta;
  int32_t* status;
};

template <bool EMBED, int NV>
__device__ __forceinline__ void load_s(const LnArgs& g, int64_t t, int lane, float4 (&v)[NV], uint32_t key) {
  if (EMBED) {
    int64_t id = g.ids[t];
    if (id < 0 || id >= g.V) {
      if (g.status && lane == 0) atomicOr(g.status, 2);
      id = 0;
    }
    const int ps = (int)(t % g.L);
    const float* w = g.word + id * g.H;
    const float* pp = g.pos + (int64_t)ps * g.H;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int c = 4 * (lane + 64 * j);
      if (c < g.H) {
        const float4 a = ld4(w + c), b = ld4(pp + c), e = ld4(g.type0 + c);
        v[j] = make_float4(a.x + b.x + e.x, a.y + b.y + e.y, a.z + b.z + e.z, a.w + b.w + e.w);
      } else {
        v[j] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
  } else {
    const float* xr = g.x + t * g.ldx;
    const float* rr = g.res + t * g.ldr;
    const uint32_t e0 = (uint32_t)(t * g.H);
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int c = 4 * (lane + 64 * j);
      if (c < g.H) {
        float4 a = ld4(xr + c);
        const float4 b = ld4(rr + c);
        if (g.p > 0.f) {
          a.x = nr_dropout_keep(key, e0 + c, g.thresh) ? a.x * g.pscale : 0.f;
          a.y = nr_dropout_keep(key, e0 + c + 1, g.thresh) ? a.y * g.pscale : 0.f;
          a.z = nr_dropout_keep(key, e0 + c + 2, g.thresh) ? a.z * g.pscale : 0.f;
          a.w = nr_dropout_keep(key, e0 + c + 3, g.thresh) ? a.w * g.pscale : 0.f;
        }
        v[j] = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
      } else {
        v[j] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
  }
}

template <bool EMBED, int NV>
__global__ void __launch_bounds__(256) ln_fwd_kernel(LnArgs g) {
  const int lane = threadIdx.x & 63;
  const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= g.T) return;
  const uint32_t key = g.rng ? nr_dropout_key(g.rng[0], g.rng[1] + g.offset) : g.key;
  float4 v[NV];
  load_s<EMBED, NV>(g, t, lane, v, key);
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NV; ++j) s += v[j].x + v[j].y + v[j].z + v[j].w;
  const float invH = 1.f / (float)g.H;
  const float mean = nr_wave_sum(s) * invH;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < NV; ++j)
    if (4 * (lane + 64 * j) < g.H) {
      const float a = v[j].x - mean, b = v[j].y - mean, c = v[j].z - mean, d = v[j].w - mean;
      q += a * a + b * b + c * c + d * d;
    }
  const float rstd = rsqrtf(nr_wave_sum(q) * invH + g.eps);
  float* orow = g.out + t * g.ldo;
  const uint32_t e0 = (uint32_t)(t * g.H);
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c = 4 * (lane + 64 * j);
    if (c >= g.H) continue;
    const float4 gm = ld4(g.gamma + c), bt = ld4(g.beta + c);
    float4 y = make_float4((v[j].x - mean) * rstd * gm.x + bt.x, (v[j].y - mean) * rstd * gm.y + bt.y,
                           (v[j].z - mean) * rstd * gm.z + bt.z, (v[j].w - mean) * rstd * gm.w + bt.w);
    if (EMBED && g.p > 0.f) {   // BertEmbeddings.dropout after the LayerNorm
      y.x = nr_dropout_keep(key, e0 + c, g.thresh) ? y.x * g.pscale : 0.f;
      y.y = nr_dropout_keep(key, e0 + c + 1, g.thresh) ? y.y * g.pscale : 0.f;
      y.z = nr_dropout_keep(key, e0 + c + 2, g.thresh) ? y.z * g.pscale : 0.f;
      y.w = nr_dropout_keep(key, e0 + c + 3, g.thresh) ? y.w * g.pscale : 0.f;
    }
    st4(orow + c, y);
  }
  if (lane == 0) {
    g.stats[2 * t] = mean;
    g.stats[2 * t + 1] = rstd;
  }
}

// The add-LN backward (!EMBED) loads the NEXT row's x, res, dout and stats into registers before the
// current row's arithmetic: a wave walks ~4 rows of the 16 k-token user sequence one after another,
// and without it each row paid its loads' full latency.
template <bool EMBED, int NV>
__global__ void __launch_bounds__(256) ln_bwd_kernel(LnArgs g) {
  __shared__ float red[4][2][256 * NV];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t key = g.rng ? nr_dropout_key(g.rng[0], g.rng[1] + g.offset) : g.key;
  float4 ag[NV], ab[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) ag[j] = ab[j] = make_float4(0.f, 0.f, 0.f, 0.f);
  const float invH = 1.f / (float)g.H;
  // one row: v = the LN input (dropout and residual applied), d = dL/d(out) as loaded
  auto row = [&](int64_t t, const float4 (&v)[NV], const float4 (&dl)[NV], float mean, float rstd) {
    const uint32_t e0 = (uint32_t)(t * g.H);
    float4 dy[NV], xh[NV];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int c = 4 * (lane + 64 * j);
      if (c >= g.H) {
        dy[j] = xh[j] = make_float4(0.f, 0.f, 0.f, 0.f);
        continue;
      }
      float4 d = dl[j];
      if (EMBED && g.p > 0.f) {
        d.x = nr_dropout_keep(key, e0 + c, g.thresh) ? d.x * g.pscale : 0.f;
        d.y = nr_dropout_keep(key, e0 + c + 1, g.thresh) ? d.y * g.pscale : 0.f;
        d.z = nr_dropout_keep(key, e0 + c + 2, g.thresh) ? d.z * g.pscale : 0.f;
        d.w = nr_dropout_keep(key, e0 + c + 3, g.thresh) ? d.w * g.pscale : 0.f;
      }
      dy[j] = d;
      xh[j] = make_float4((v[j].x - mean) * rstd, (v[j].y - mean) * rstd, (v[j].z - mean) * rstd,
                          (v[j].w - mean) * rstd);
      const float4 gm = ld4(g.gamma + c);
      const float4 dh = make_float4(d.x * gm.x, d.y * gm.y, d.z * gm.z, d.w * gm.w);
      s1 += dh.x + dh.y + dh.z + dh.w;
      s2 += dh.x * xh[j].x + dh.y * xh[j].y + dh.z * xh[j].z + dh.w * xh[j].w;
      ag[j].x += d.x * xh[j].x; ag[j].y += d.y * xh[j].y; ag[j].z += d.z * xh[j].z; ag[j].w += d.w * xh[j].w;
      ab[j].x += d.x; ab[j].y += d.y; ab[j].z += d.z; ab[j].w += d.w;
    }
    const float m1 = nr_wave_sum(s1) * invH, m2 = nr_wave_sum(s2) * invH;
    float* srow = g.ds + t * g.ldds;
    float* xrow = EMBED ? nullptr : g.dx + t * g.lddx;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int c = 4 * (lane + 64 * j);
      if (c >= g.H) continue;
      const float4 gm = ld4(g.gamma + c);
      const float4 gs = make_float4(rstd * (dy[j].x * gm.x - m1 - xh[j].x * m2),
                                    rstd * (dy[j].y * gm.y - m1 - xh[j].y * m2),
                                    rstd * (dy[j].z * gm.z - m1 - xh[j].z * m2),
                                    rstd * (dy[j].w * gm.w - m1 - xh[j].w * m2));
      st4(srow + c, gs);
      if (!EMBED) {   // d(dense) = dropout mask * scale * gs
        float4 dx = gs;
        if (g.p > 0.f) {
          dx.x = nr_dropout_keep(key, e0 + c, g.thresh) ? dx.x * g.pscale : 0.f;
          dx.y = nr_dropout_keep(key, e0 + c + 1, g.thresh) ? dx.y * g.pscale : 0.f;
          dx.z = nr_dropout_keep(key, e0 + c + 2, g.thresh) ? dx.z * g.pscale : 0.f;
          dx.w = nr_dropout_keep(key, e0 + c + 3, g.thresh) ? dx.w * g.pscale : 0.f;
        }
        st4(xrow + c, dx);
      }
    }
  };
  const int64_t stride = (int64_t)gridDim.x * 4;
  if constexpr (EMBED) {
    for (int64_t t = (int64_t)blockIdx.x * 4 + wave; t < g.T; t += stride) {
      float4 v[NV], dl[NV];
      load_s<EMBED, NV>(g, t, lane, v, key);
      const float* drow = g.dout + t * g.ldd;
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        const int c = 4 * (lane + 64 * j);
        dl[j] = c < g.H ? ld4(drow + c) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
      row(t, v, dl, g.stats[2 * t], g.stats[2 * t + 1]);
    }
  } else {
    float4 xn[NV], rn[NV], dn[NV];
    float mn = 0.f, sn = 0.f;
    auto fetch = [&](int64_t t) {
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        const int c = 4 * (lane + 64 * j);
        if (c < g.H) {
          xn[j] = ld4(g.x + t * g.ldx + c);
          rn[j] = ld4(g.res + t * g.ldr + c);
          dn[j] = ld4(g.dout + t * g.ldd + c);
        } else {
          xn[j] = rn[j] = dn[j] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
      mn = g.stats[2 * t];
      sn = g.stats[2 * t + 1];
    };
    int64_t t = (int64_t)blockIdx.x * 4 + wave;
    if (t < g.T) fetch(t);
    for (; t < g.T; t += stride) {
      float4 v[NV], dl[NV];
      const uint32_t e0 = (uint32_t)(t * g.H);
#pragma unroll
      for (int j = 0; j < NV; ++j) {   // load_s's arithmetic on the prefetched row
        const int c = 4 * (lane + 64 * j);
        float4 a = xn[j];
        const float4 b = rn[j];
        if (c < g.H && g.p > 0.f) {
          a.x = nr_dropout_keep(key, e0 + c, g.thresh) ? a.x * g.pscale : 0.f;
          a.y = nr_dropout_keep(key, e0 + c + 1, g.thresh) ? a.y * g.pscale : 0.f;
          a.z = nr_dropout_keep(key, e0 + c + 2, g.thresh) ? a.z * g.pscale : 0.f;
          a.w = nr_dropout_keep(key, e0 + c + 3, g.thresh) ? a.w * g.pscale : 0.f;
        }
        v[j] = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
        dl[j] = dn[j];
      }
      const float mean = mn, rstd = sn;
      if (t + stride < g.T) fetch(t + stride);
      row(t, v, dl, mean, rstd);
    }
  }
  // dgamma / dbeta: per-wave partials -> LDS -> one atomic per column per workgroup
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c = 4 * (lane + 64 * j);
    red[wave][0][c] = ag[j].x; red[wave][0][c + 1] = ag[j].y; red[wave][0][c + 2] = ag[j].z; red[wave][0][c + 3] = ag[j].w;
    red[wave][1][c] = ab[j].x; red[wave][1][c + 1] = ab[j].y; red[wave][1][c + 2] = ab[j].z; red[wave][1][c + 3] = ab[j].w;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < g.H; c += 256) {
    atomicAdd(g.dgamma + c, red[0][0][c] + red[1][0][c] + red[2][0][c] + red[3][0][c]);
    atomicAdd(g.dbeta + c, red[0][1][c] + red[1][1][c] + red[2][1][c] + red[3][1][c]);
  }
}

// the backward's grid-stride launch: at most one round of resident workgroups (CUs x occupancy of this
// instantiation, cached per device), at most 1024 -- each workgroup ends in one dgamma / dbeta atomic per
// column, and a second round would run the last rows' workgroups on an otherwise idle chip
template <bool EMBED, int NV>
unsigned ln_bwd_grid(int64_t T) {
  static int cap[16] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) dev = 0;
  if (cap[dev] == 0) {
    int cus = 0, per = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, ln_bwd_kernel<EMBED, NV>, 256, 0) != hipSuccess || per < 1)
      per = 1;
    cap[dev] = cus * per < 1024 ? cus * per : 1024;
  }
  const int64_t nb = (T + 3) / 4;
  return (unsigned)(nb < cap[dev] ? nb : cap[dev]);
}

template <bool EMBED, bool BWD>
int launch_ln(const LnArgs& g, hipStream_t s) {
  if (g.T == 0) return NR_OK;
  const int nv = (g.H + 255) / 256;
  const dim3 grid((unsigned)((g.T + 3) / 4));
#define NR_LN(NV)                                                                                    \
  if (nv == NV) {                                                                                    \
    if (BWD) hipLaunchKernelGGL((ln_bwd_kernel<EMBED, NV>), dim3(ln_bwd_grid<EMBED, NV>(g.T)), dim3(256), 0, s, g); \
    else hipLaunchKernelGGL((ln_fwd_kernel<EMBED, NV>), grid, dim3(256), 0, s, g);                   \
  }
  NR_LN(1) else NR_LN(2) else NR_LN(3) else NR_LN(4) else return NR_EINVAL(9);
#undef NR_LN
  NR_LAUNCH_CHECK();
  return NR_OK;
}

void set_drop(LnArgs& g, float p, uint64_t seed, uint64_t offset, const uint64_t* rng) {
  g.p = p;
  g.pscale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  g.thresh = nr_dropout_threshold(p);
  g.key = nr_dropout_key(seed, offset);
  g.rng = rng;
  g.offset = offset;
}

// ------------------------------------------------------------------------------------ attention

struct AttnArgs {
  const float* qkv; int64_t ldq; int64_t koff, voff;   // Q at col head*64, K at koff + head*64, V at voff + ...
  const void* mask; int mdt;
  int64_t nseq; int L; int heads; int chunks;
  float p; float pscale; uint32_t thresh; uint32_t key; const uint64_t* rng; uint64_t offset;
  float* ctx; int64_t ldc;          // fwd output
  float* ml;                        // [T][heads][2] = (max, 1/sum) per query
  const float* dctx; int64_t ldd;   // bwd: upstream grad of ctx
  const float* Dq;                  // bwd: [T][heads] rowsum(dctx * ctx)
  float* dqkv; int64_t lddq;        // bwd output (same column layout as qkv)
  // dropout keep bits (optional): word ((seq * heads + head) * L + q) * nkb + kb holds query q's 32 keys
  // of key tile kb, bit r + 16 h = key kb * 32 + crow(r, h) (the forward lane's own 16 bits per half);
  // the bf16-MFMA forward stores them, both backward kernels read them instead of re-hashing
  uint32_t* keep; int nkb;
  // bwd, four-wave launches (L > 96): dS = P (dP' - D) as attn_bwd_kv_mp_kernel forms it, row
  // ((seq * heads + head) * nkb + kb) * 32 nkb + q holding query q's 32 keys of key tile kb (128 B;
  // queries padded to 32 nkb so the stores need no bound);
  // attn_bwd_q_ds_kernel reads it back instead of recomputing S, P and dP
  float* dsb;
};

__device__ __forceinline__ int64_t keep_word(const AttnArgs& g, int64_t seq, int head, int q, int kb) {
  return ((seq * g.heads + head) * (int64_t)g.L + q) * g.nkb + kb;
}

__device__ __forceinline__ uint32_t attn_key(const AttnArgs& g, int64_t seq, int head) {
  const uint32_t k = g.rng ? nr_dropout_key(g.rng[0], g.rng[1] + g.offset) : g.key;
  return nr_hash32(k ^ (uint32_t)((seq * g.heads + head) * 0x85EBCA6Bull));
}

// stage rows r0 .. r0+31 of two 64-wide column blocks into LDS (zeros beyond L)
__device__ __forceinline__ void stage2(float (*A)[kLS], float (*B)[kLS], const float* base, int64_t ld, int64_t row0,
                                       int r0, int L, int64_t ca, int64_t cb) {
  for (int f = threadIdx.x; f < 512; f += blockDim.x) {
    const int r = f >> 4, cc = (f & 15) * 4;
    const int j = r0 + r;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
    if (j < L) {
      const float* p = base + (row0 + j) * ld;
      a = ld4(p + ca + cc);
      b = ld4(p + cb + cc);
    }
    st4(&A[r][cc], a);
    st4(&B[r][cc], b);
  }
}

template <bool DROP>
__global__ void __launch_bounds__(256) attn_fwd_kernel(AttnArgs g) {
  __shared__ float Ks[32][kLS];
  __shared__ float Vs[32][kLS];
  __shared__ float kadd[32];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 31, hh = lane >> 5;
  const int nw = blockDim.x >> 6;
  int64_t bid = blockIdx.x;
  const int qc = (int)(bid % g.chunks);
  bid /= g.chunks;
  const int head = (int)(bid % g.heads);
  const int64_t seq = bid / g.heads;
  const int L = g.L;
  const int64_t row0 = seq * L;
  const int q0 = (qc * nw + wave) * 32;
  const bool active = q0 < L;
  const int q = q0 + c;
  const uint32_t dkey = DROP ? attn_key(g, seq, head) : 0u;

  float qf[32];   // B operand of Sᵀ = K Qᵀ: Q[q][32 hh + s] / 8 (exact power-of-two scale)
  if (active && q < L) {
    const float* qp = g.qkv + (row0 + q) * g.ldq + head * kHD + 32 * hh;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float4 x = ld4(qp + 4 * j);
      qf[4 * j] = x.x * 0.125f; qf[4 * j + 1] = x.y * 0.125f; qf[4 * j + 2] = x.z * 0.125f; qf[4 * j + 3] = x.w * 0.125f;
    }
  } else {
#pragma unroll
    for (int j = 0; j < 32; ++j) qf[j] = 0.f;
  }
  f32x16 o0, o1;
#pragma unroll
  for (int r = 0; r < 16; ++r) o0[r] = o1[r] = 0.f;
  float m = -INFINITY, l = 0.f;
  const int nkb = (L + 31) / 32;
  for (int kb = 0; kb < nkb; ++kb) {
    __syncthreads();
    stage2(Ks, Vs, g.qkv, g.ldq, row0, kb * 32, L, g.koff + head * kHD, g.voff + head * kHD);
    if (threadIdx.x < 32) {
      const int j = kb * 32 + threadIdx.x;
      kadd[threadIdx.x] = j >= L ? -INFINITY : (nr_mask_at(g.mask, g.mdt, row0 + j) ? 0.f : kNegMax);
    }
    __syncthreads();
    if (!active) continue;
    f32x16 s;
#pragma unroll
    for (int r = 0; r < 16; ++r) s[r] = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float4 a = ld4(&Ks[c][32 * hh + 4 * j]);
      s = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, qf[4 * j], s, 0, 0, 0);
      s = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, qf[4 * j + 1], s, 0, 0, 0);
      s = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, qf[4 * j + 2], s, 0, 0, 0);
      s = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, qf[4 * j + 3], s, 0, 0, 0);
    }
    float mx = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      s[r] = s[r] + kadd[crow(r, hh)];
      mx = fmaxf(mx, s[r]);
    }
    mx = xhalf_max(mx);
    const float mn = fmaxf(m, mx);
    const float alpha = __expf(m - mn);
    float ps = 0.f;
    float pe[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      pe[r] = __expf(s[r] - mn);
      ps += pe[r];
    }
    ps = xhalf_sum(ps);
    l = l * alpha + ps;
    m = mn;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      o0[r] *= alpha;
      o1[r] *= alpha;
    }
    if (DROP) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const uint32_t e = (uint32_t)q * (uint32_t)L + (uint32_t)(kb * 32 + crow(r, hh));
        pe[r] = nr_dropout_keep(dkey, e, g.thresh) ? pe[r] * g.pscale : 0.f;
      }
    }
#pragma unroll
    for (int st = 0; st < 16; ++st) {
      const int kr = crow(st, hh);
      o0 = __builtin_amdgcn_mfma_f32_32x32x2f32(Vs[kr][c], pe[st], o0, 0, 0, 0);
      o1 = __builtin_amdgcn_mfma_f32_32x32x2f32(Vs[kr][32 + c], pe[st], o1, 0, 0, 0);
    }
  }
  if (!active || q >= L) return;
  const float inv = 1.f / l;
  float* op = g.ctx + (row0 + q) * g.ldc + head * kHD;
#pragma unroll
  for (int gq = 0; gq < 4; ++gq) {
    const int d = 8 * gq + 4 * hh;
    st4(op + d, make_float4(o0[4 * gq] * inv, o0[4 * gq + 1] * inv, o0[4 * gq + 2] * inv, o0[4 * gq + 3] * inv));
    st4(op + 32 + d, make_float4(o1[4 * gq] * inv, o1[4 * gq + 1] * inv, o1[4 * gq + 2] * inv, o1[4 * gq + 3] * inv));
  }
  if (hh == 0) {
    float* mp = g.ml + ((row0 + q) * g.heads + head) * 2;
    mp[0] = m;
    mp[1] = inv;
  }
}

// D[t][h] = Σ_d dctx[t][h*64+d] * ctx[t][h*64+d]   (one thread per (token, head))
// D[t][h] = dctx[t, h-th 64 columns] . ctx[t, same]: one float4 of one token per thread (coalesced
// rows), the 16 lanes of a head's 64 columns reduced by shuffles (was one thread per (token, head)
// reading its 256-B slices: 64 cache lines per wave instruction, 2.3 TB/s on the user sequence)
__global__ void __launch_bounds__(256) attn_dsum_kernel(const float* dctx, int64_t ldd, const float* ctx, int64_t ldc,
                                                        int64_t T, int heads, float* D) {
  const int c4 = heads * (kHD / 4);   // float4 per token row
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t t = i / c4;
  const int c = (int)(i - t * c4);
  float s = 0.f;
  if (t < T) {
    const float4 x = ld4(dctx + t * ldd + 4 * c), y = ld4(ctx + t * ldc + 4 * c);
    s = x.x * y.x + x.y * y.y + x.z * y.z + x.w * y.w;
  }
  // a head's 16 float4 are 16 consecutive threads (c4 is a multiple of 16, so they share a wave)
#pragma unroll
  for (int d = 8; d >= 1; d >>= 1) s += __shfl_xor(s, d, 64);
  if (t < T && (c & 15) == 0) D[t * heads + (c >> 4)] = s;
}

// dK, dV: a wave owns 32 keys; query tiles (Q, dctx, stats) staged in LDS.
template <bool DROP>
__global__ void __launch_bounds__(256) attn_bwd_kv_kernel(AttnArgs g) {
  __shared__ float Qs[32][kLS];
  __shared__ float Os[32][kLS];   // dctx tile
  __shared__ float qm[32], qi[32], qd[32];
  __shared__ __attribute__((aligned(16))) uint32_t kwd[4][32];   // per wave: the tile's 32 queries' words of its key tile
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 31, hh = lane >> 5;
  const int nw = blockDim.x >> 6;
  int64_t bid = blockIdx.x;
  const int kc = (int)(bid % g.chunks);
  bid /= g.chunks;
  const int head = (int)(bid % g.heads);
  const int64_t seq = bid / g.heads;
  const int L = g.L;
  const int64_t row0 = seq * L;
  const int k0 = (kc * nw + wave) * 32;
  const bool active = k0 < L;
  const int key = k0 + c;
  const uint32_t dkey = DROP ? attn_key(g, seq, head) : 0u;

  float kf[32], vf[32];
  float kadd = -INFINITY;
  if (active && key < L) {
    const float* kp = g.qkv + (row0 + key) * g.ldq + g.koff + head * kHD + 32 * hh;
    const float* vp = g.qkv + (row0 + key) * g.ldq + g.voff + head * kHD + 32 * hh;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float4 x = ld4(kp + 4 * j), y = ld4(vp + 4 * j);
      kf[4 * j] = x.x * 0.125f; kf[4 * j + 1] = x.y * 0.125f; kf[4 * j + 2] = x.z * 0.125f; kf[4 * j + 3] = x.w * 0.125f;
      vf[4 * j] = y.x; vf[4 * j + 1] = y.y; vf[4 * j + 2] = y.z; vf[4 * j + 3] = y.w;
    }
    kadd = nr_mask_at(g.mask, g.mdt, row0 + key) ? 0.f : kNegMax;
  } else {
#pragma unroll
    for (int j = 0; j < 32; ++j) kf[j] = vf[j] = 0.f;
  }
  f32x16 dk0, dk1, dv0, dv1;
#pragma unroll
  for (int r = 0; r < 16; ++r) dk0[r] = dk1[r] = dv0[r] = dv1[r] = 0.f;
  const int nqb = (L + 31) / 32;
  for (int qb = 0; qb < nqb; ++qb) {
    __syncthreads();
    for (int f = threadIdx.x; f < 512; f += blockDim.x) {   // Q and dctx rows of the query tile
      const int r = f >> 4, cc = (f & 15) * 4;
      const int j = qb * 32 + r;
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
      if (j < L) {
        a = ld4(g.qkv + (row0 + j) * g.ldq + head * kHD + cc);
        b = ld4(g.dctx + (row0 + j) * g.ldd + head * kHD + cc);
      }
      st4(&Qs[r][cc], a);
      st4(&Os[r][cc], b);
    }
    if (threadIdx.x < 32) {
      const int j = qb * 32 + threadIdx.x;
      if (j < L) {
        const float* mp = g.ml + ((row0 + j) * g.heads + head) * 2;
        qm[threadIdx.x] = mp[0];
        qi[threadIdx.x] = mp[1];
        qd[threadIdx.x] = g.Dq[(row0 + j) * g.heads + head];
      } else {
        qm[threadIdx.x] = INFINITY;   // exp(s - inf) = 0: no such query
        qi[threadIdx.x] = 0.f;
        qd[threadIdx.x] = 0.f;
      }
    }
    __syncthreads();
    if (!active) continue;
    f32x16 s, dp;
#pragma unroll
    for (int r = 0; r < 16; ++r) s[r] = dp[r] = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float4 a = ld4(&Qs[c][32 * hh + 4 * j]);
      const float4 b = ld4(&Os[c][32 * hh + 4 * j]);
      s = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, kf[4 * j], s, 0, 0, 0);
      s = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, kf[4 * j + 1], s, 0, 0, 0);
      s = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, kf[4 * j + 2], s, 0, 0, 0);
      s = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, kf[4 * j + 3], s, 0, 0, 0);
      dp = __builtin_amdgcn_mfma_f32_32x32x2f32(b.x, vf[4 * j], dp, 0, 0, 0);
      dp = __builtin_amdgcn_mfma_f32_32x32x2f32(b.y, vf[4 * j + 1], dp, 0, 0, 0);
      dp = __builtin_amdgcn_mfma_f32_32x32x2f32(b.z, vf[4 * j + 2], dp, 0, 0, 0);
      dp = __builtin_amdgcn_mfma_f32_32x32x2f32(b.w, vf[4 * j + 3], dp, 0, 0, 0);
    }
    // S rows = queries crow(r, hh) of the tile, column = this lane's key
    float pd[16], ds[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int qr = crow(r, hh);
      const float pr = __expf(s[r] + kadd - qm[qr]) * qi[qr];
      float d = dp[r];
      float pdr = pr;
      if (DROP) {
        const uint32_t e = (uint32_t)(qb * 32 + qr) * (uint32_t)L + (uint32_t)key;
        const bool kp = nr_dropout_keep(dkey, e, g.thresh);
        d = kp ? d * g.pscale : 0.f;
        pdr = kp ? pr * g.pscale : 0.f;
      }
      pd[r] = pdr;
      ds[r] = pr * (d - qd[qr]);
    }
#pragma unroll
    for (int st = 0; st < 16; ++st) {
      const int qr = crow(st, hh);
      dv0 = __builtin_amdgcn_mfma_f32_32x32x2f32(Os[qr][c], pd[st], dv0, 0, 0, 0);
      dv1 = __builtin_amdgcn_mfma_f32_32x32x2f32(Os[qr][32 + c], pd[st], dv1, 0, 0, 0);
      dk0 = __builtin_amdgcn_mfma_f32_32x32x2f32(Qs[qr][c], ds[st], dk0, 0, 0, 0);
      dk1 = __builtin_amdgcn_mfma_f32_32x32x2f32(Qs[qr][32 + c], ds[st], dk1, 0, 0, 0);
    }
  }
  if (!active || key >= L) return;
  float* kp = g.dqkv + (row0 + key) * g.lddq + g.koff + head * kHD;
  float* vp = g.dqkv + (row0 + key) * g.lddq + g.voff + head * kHD;
#pragma unroll
  for (int gq = 0; gq < 4; ++gq) {
    const int d = 8 * gq + 4 * hh;
    st4(kp + d, make_float4(dk0[4 * gq] * 0.125f, dk0[4 * gq + 1] * 0.125f, dk0[4 * gq + 2] * 0.125f,
                            dk0[4 * gq + 3] * 0.125f));
    st4(kp + 32 + d, make_float4(dk1[4 * gq] * 0.125f, dk1[4 * gq + 1] * 0.125f, dk1[4 * gq + 2] * 0.125f,
                                 dk1[4 * gq + 3] * 0.125f));
    st4(vp + d, make_float4(dv0[4 * gq], dv0[4 * gq + 1], dv0[4 * gq + 2], dv0[4 * gq + 3]));
    st4(vp + 32 + d, make_float4(dv1[4 * gq], dv1[4 * gq + 1], dv1[4 * gq + 2], dv1[4 * gq + 3]));
  }
}

// dQ: a wave owns 32 queries; key tiles staged in LDS; scores transposed (query on the lane).
template <bool DROP>
__global__ void __launch_bounds__(256) attn_bwd_q_kernel(AttnArgs g) {
  __shared__ float Ks[32][kLS];
  __shared__ float Vs[32][kLS];
  __shared__ float kadd[32];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 31, hh = lane >> 5;
  const int nw = blockDim.x >> 6;
  int64_t bid = blockIdx.x;
  const int qc = (int)(bid % g.chunks);
  bid /= g.chunks;
  const int head = (int)(bid % g.heads);
  const int64_t seq = bid / g.heads;
  const int L = g.L;
  const int64_t row0 = seq * L;
  const int q0 = (qc * nw + wave) * 32;
  const bool active = q0 < L;
  const int q = q0 + c;
  const uint32_t dkey = DROP ? attn_key(g, seq, head) : 0u;

  float qf[32], df[32];
  float mq = INFINITY, iq = 0.f, dq = 0.f;
  if (active && q < L) {
    const float* qp = g.qkv + (row0 + q) * g.ldq + head * kHD + 32 * hh;
    const float* op = g.dctx + (row0 + q) * g.ldd + head * kHD + 32 * hh;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float4 x = ld4(qp + 4 * j), y = ld4(op + 4 * j);
      qf[4 * j] = x.x * 0.125f; qf[4 * j + 1] = x.y * 0.125f; qf[4 * j + 2] = x.z * 0.125f; qf[4 * j + 3] = x.w * 0.125f;
      df[4 * j] = y.x; df[4 * j + 1] = y.y; df[4 * j + 2] = y.z; df[4 * j + 3] = y.w;
    }
    const float* mp = g.ml + ((row0 + q) * g.heads + head) * 2;
    mq = mp[0];
    iq = mp[1];
    dq = g.Dq[(row0 + q) * g.heads + head];
  } else {
#pragma unroll
    for (int j = 0; j < 32; ++j) qf[j] = df[j] = 0.f;
  }
  f32x16 a0, a1;
#pragma unroll
  for (int r = 0; r < 16; ++r) a0[r] = a1[r] = 0.f;
  const int nkb = (L + 31) / 32;
  for (int kb = 0; kb < nkb; ++kb) {
    __syncthreads();
    stage2(Ks, Vs, g.qkv, g.ldq, row0, kb * 32, L, g.koff + head * kHD, g.voff + head * kHD);
    if (threadIdx.x < 32) {
      const int j = kb * 32 + threadIdx.x;
      kadd[threadIdx.x] = j >= L ? -INFINITY : (nr_mask_at(g.mask, g.mdt, row0 + j) ? 0.f : kNegMax);
    }
    __syncthreads();
    if (!active) continue;
    f32x16 s, dp;
#pragma unroll
    for (int r = 0; r < 16; ++r) s[r] = dp[r] = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float4 a = ld4(&Ks[c][32 * hh + 4 * j]);
      const float4 b = ld4(&Vs[c][32 * hh + 4 * j]);
      s = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, qf[4 * j], s, 0, 0, 0);
      s = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, qf[4 * j + 1], s, 0, 0, 0);
      s = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, qf[4 * j + 2], s, 0, 0, 0);
      s = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, qf[4 * j + 3], s, 0, 0, 0);
      dp = __builtin_amdgcn_mfma_f32_32x32x2f32(b.x, df[4 * j], dp, 0, 0, 0);
      dp = __builtin_amdgcn_mfma_f32_32x32x2f32(b.y, df[4 * j + 1], dp, 0, 0, 0);
      dp = __builtin_amdgcn_mfma_f32_32x32x2f32(b.z, df[4 * j + 2], dp, 0, 0, 0);
      dp = __builtin_amdgcn_mfma_f32_32x32x2f32(b.w, df[4 * j + 3], dp, 0, 0, 0);
    }
    float ds[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int kr = crow(r, hh);
      const float pr = __expf(s[r] + kadd[kr] - mq) * iq;
      float d = dp[r];
      if (DROP) {
        const uint32_t e = (uint32_t)q * (uint32_t)L + (uint32_t)(kb * 32 + kr);
        d = nr_dropout_keep(dkey, e, g.thresh) ? d * g.pscale : 0.f;
      }
      ds[r] = pr * (d - dq);
    }
#pragma unroll
    for (int st = 0; st < 16; ++st) {
      const int kr = crow(st, hh);
      a0 = __builtin_amdgcn_mfma_f32_32x32x2f32(Ks[kr][c], ds[st], a0, 0, 0, 0);
      a1 = __builtin_amdgcn_mfma_f32_32x32x2f32(Ks[kr][32 + c], ds[st], a1, 0, 0, 0);
    }
  }
  if (!active || q >= L) return;
  float* op = g.dqkv + (row0 + q) * g.lddq + head * kHD;
#pragma unroll
  for (int gq = 0; gq < 4; ++gq) {
    const int d = 8 * gq + 4 * hh;
    st4(op + d, make_float4(a0[4 * gq] * 0.125f, a0[4 * gq + 1] * 0.125f, a0[4 * gq + 2] * 0.125f,
                            a0[4 * gq + 3] * 0.125f));
    st4(op + 32 + d, make_float4(a1[4 * gq] * 0.125f, a1[4 * gq + 1] * 0.125f, a1[4 * gq + 2] * 0.125f,
                                 a1[4 * gq + 3] * 0.125f));
  }
}

// ---- attention products on the bf16 MFMA (prec = NR_GEMM_BF16X6 / NR_GEMM_BF16) -----------------
// The f32 kernels above run v_mfma_f32_32x32x2_f32; these run the same products on
// v_mfma_f32_32x32x16_bf16 in the caller's GEMM arithmetic (mfma_planes.h: NP = 3 is bf16x6, the
// fp32-class six-product form at 2.7x the f32 MFMA's rate; NP = 1 plain bf16).  One 16-deep step
// feeds lane (c, h) eight k-slots 8h .. 8h + 7:
//   * head-dim contractions (S = Q Kᵀ, dP = dctx Vᵀ): step t gives slot 8h + u the dim 32h + 8t + u,
//     the f32 form's per-lane half-row -- the wave's own rows are split once into planes, the tile's
//     rows come split from LDS (row-major plane image, rowfrag);
//   * tile-row contractions (O = P V, dV = Pᵀ dctx, dK = dSᵀ Q, dQ = dS K): step t gives slot u of
//     lane (c, h) the tile row crow(8t + u, h) -- the row the accumulator value the lane already
//     holds belongs to -- so the tile is staged TRANSPOSED (dims x rows) and read as two 4-row runs
//     per plane (colfrag).
// Every staged element is split once per tile by the staging threads, not once per wave.
// compile-time A/B knob (tools/build_ab.sh): the dK/dV pass of four-wave sequences as eight-wave workgroups
#ifndef NR_ATTN_BWD_W8
#define NR_ATTN_BWD_W8 1
#endif
constexpr bool kNrAttnBwdW8 = NR_ATTN_BWD_W8;
constexpr int kKR = kHD + 8;   // row-major plane row: 64 dims + 8 pad (144 B: ds_read_b128 conflict-free)
constexpr int kVR = 36;        // transposed plane row: 32 rows + 4 pad (72 B: ds_read_b64 conflict-free)

template <int NP>
__device__ __forceinline__ void put4(uint16_t (*P)[32][kKR], int r, int cc, float4 a) {
  if constexpr (NP == 1) {
    *reinterpret_cast<uint2*>(&P[0][r][cc]) = make_uint2(nrfast::pk_bf16(a.x, a.y), nrfast::pk_bf16(a.z, a.w));
  } else {
    uint2 p0, p1, p2;
    nrfast::split4(a.x, a.y, a.z, a.w, p0, p1, p2);
    *reinterpret_cast<uint2*>(&P[0][r][cc]) = p0;
    *reinterpret_cast<uint2*>(&P[1][r][cc]) = p1;
    *reinterpret_cast<uint2*>(&P[2][r][cc]) = p2;
  }
}

template <int NP>
__device__ __forceinline__ void put2(uint16_t (*T)[kHD][kVR], int d, int k, float a, float b) {
  if constexpr (NP == 1) {
    *reinterpret_cast<uint32_t*>(&T[0][d][k]) = nrfast::pk_bf16(a, b);
  } else {
    uint32_t h2, m2, l2;
    nrfast::split2(a, b, h2, m2, l2);
    *reinterpret_cast<uint32_t*>(&T[0][d][k]) = h2;
    *reinterpret_cast<uint32_t*>(&T[1][d][k]) = m2;
    *reinterpret_cast<uint32_t*>(&T[2][d][k]) = l2;
  }
}

// Staging slot of thread f (0..255): rows 2 kp, 2 kp + 1 and dims 4 dq .. 4 dq + 3 of the tile, with
// f's bits dealt as kp = {f0, f1, f4, f6}, dq = {f2, f3, f5, f7} so that both images are written
// conflict-free: a ds_write_b64 group (16 lanes) of the row-major image covers kp mod 4 x dq mod 4 =
// 16 distinct bank pairs of a 36-dword row stride, a ds_write_b32 group (32 lanes) of the transposed
// one 8 dq + kp = 32 distinct banks of an 18-dword row stride.  (kp = f & 15 put four lanes of a
// b64 group on each bank pair: the attention kernels' 2.5 - 3.2 conflict cycles per LDS instruction,
// profiles/r04_j_pmc_xf_attn_*.json.)
__device__ __forceinline__ void tile_slot(int f, int& kp, int& dq) {
  kp = (f & 3) | ((f >> 2) & 4) | ((f >> 3) & 8);
  dq = ((f >> 2) & 3) | ((f >> 3) & 4) | ((f >> 4) & 8);
}

// Stage rows j0 .. j0 + 31 (zeros at and past L) of one 64-wide column block, split into planes,
// row-major into P and/or transposed into T; the whole workgroup takes part.
template <int NP>
__device__ __forceinline__ void stage_planes(uint16_t (*P)[32][kKR], uint16_t (*T)[kHD][kVR], const float* base,
                                             int64_t ld, int64_t row0, int j0, int L, int64_t col) {
  const int tid = threadIdx.x;
  if (NP == 3 && P && T) {
    // (workgroups of fewer than four waves, e.g. the 30-token titles)
    // both images from one load and one split per element: a thread takes rows 2 kp, 2 kp + 1 and
    // dims 4 dq .. 4 dq + 3, stores their row-major quads and repacks the same bf16 halves into the
    // transposed (dim, row pair) words
    for (int f = tid; f < 256; f += blockDim.x) {
      int kp, dq;
      tile_slot(f, kp, dq);
      const int j = j0 + 2 * kp;
      const float* vb = base + (row0 + j) * ld + col + 4 * dq;
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
      if (j < L) a = ld4(vb);
      if (j + 1 < L) b = ld4(vb + ld);
      uint2 pa[3], pb[3];
      nrfast::split4(a.x, a.y, a.z, a.w, pa[0], pa[1], pa[2]);
      nrfast::split4(b.x, b.y, b.z, b.w, pb[0], pb[1], pb[2]);
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        *reinterpret_cast<uint2*>(&P[q][2 * kp][4 * dq]) = pa[q];
        *reinterpret_cast<uint2*>(&P[q][2 * kp + 1][4 * dq]) = pb[q];
        *reinterpret_cast<uint32_t*>(&T[q][4 * dq][2 * kp]) = (pa[q].x & 0xffffu) | (pb[q].x << 16);
        *reinterpret_cast<uint32_t*>(&T[q][4 * dq + 1][2 * kp]) = (pa[q].x >> 16) | (pb[q].x & 0xffff0000u);
        *reinterpret_cast<uint32_t*>(&T[q][4 * dq + 2][2 * kp]) = (pa[q].y & 0xffffu) | (pb[q].y << 16);
        *reinterpret_cast<uint32_t*>(&T[q][4 * dq + 3][2 * kp]) = (pa[q].y >> 16) | (pb[q].y & 0xffff0000u);
      }
    }
    return;
  }
  if (P) {
    for (int f = tid; f < 512; f += blockDim.x) {
      const int r = f >> 4, cc = (f & 15) * 4;
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
      if (j0 + r < L) a = ld4(base + (row0 + j0 + r) * ld + col + cc);
      put4<NP>(P, r, cc, a);
    }
  }
  if (T) {
    for (int f = tid; f < 256; f += blockDim.x) {
      int kp, dq;   // rows 2 kp, 2 kp + 1; dims 4 dq .. 4 dq + 3
      tile_slot(f, kp, dq);
      const int j = j0 + 2 * kp;
      const float* vb = base + (row0 + j) * ld + col + 4 * dq;
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
      if (j < L) a = ld4(vb);
      if (j + 1 < L) b = ld4(vb + ld);
      put2<NP>(T, 4 * dq, 2 * kp, a.x, b.x);
      put2<NP>(T, 4 * dq + 1, 2 * kp, a.y, b.y);
      put2<NP>(T, 4 * dq + 2, 2 * kp, a.z, b.z);
      put2<NP>(T, 4 * dq + 3, 2 * kp, a.w, b.w);
    }
  }
}

// head-dim step t of tile row c: dims 32 h + 8 t .. + 7 of a row-major plane image
template <int NP>
__device__ __forceinline__ Planes<NP> rowfrag(const uint16_t (*P)[32][kKR], int c, int h, int t) {
  Planes<NP> r;
#pragma unroll
  for (int p = 0; p < NP; ++p) r.v[p] = *reinterpret_cast<const bf16x8*>(&P[p][c][32 * h + 8 * t]);
  return r;
}

// tile-row step t of dim d: rows crow(8t + u, h), u = 0..7 = runs 16t + 4h .. +3 and 16t + 8 + 4h .. +3
template <int NP>
__device__ __forceinline__ Planes<NP> colfrag(const uint16_t (*T)[kHD][kVR], int d, int h, int t) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  Planes<NP> r;
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const uint2 a0 = *reinterpret_cast<const uint2*>(&T[p][d][16 * t + 4 * h]);
    const uint2 a1 = *reinterpret_cast<const uint2*>(&T[p][d][16 * t + 8 + 4 * h]);
    r.v[p] = __builtin_bit_cast(bf16x8, (u32x4){a0.x, a0.y, a1.x, a1.y});
  }
  return r;
}

// a wave's own 32-value half-row (dims 32 h .. 32 h + 31 of one row, times `scale`) as four
// head-dim steps of planes; zeros when the row does not exist
template <int NP>
__device__ __forceinline__ void own_rows(Planes<NP> (&out)[4], const float* p, bool ok, float scale) {
  float f[32];
  if (ok) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float4 x = ld4(p + 4 * j);
      f[4 * j] = x.x * scale; f[4 * j + 1] = x.y * scale; f[4 * j + 2] = x.z * scale; f[4 * j + 3] = x.w * scale;
    }
  } else {
#pragma unroll
    for (int j = 0; j < 32; ++j) f[j] = 0.f;
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) out[t] = planes8<NP>(f + 8 * t);
}

// Register-prefetched staging (workgroups of four waves): thread f holds rows 2 kp, 2 kp + 1 and dims
// 4 dq .. 4 dq + 3 (tile_slot) of the NEXT tile of one tensor, loaded while the current
// tile's products run, and writes both plane images of it from one split after the barrier.  Without
// it every tile paid a full load latency between its two barriers (one to three waves per SIMD
// cannot hide it): XFormer train step 74.3 -> 71.3 ms (profiles/r04_h_xf_*.json, same box).
template <int NP>
struct TileFetch {
  float4 a, b;
  __device__ __forceinline__ void fetch(const float* base, int64_t ld, int64_t row0, int j0, int L, int64_t col) {
    int kp, dq;
    tile_slot(threadIdx.x, kp, dq);
    const int j = j0 + 2 * kp;
    const float* vb = base + (row0 + j) * ld + col + 4 * dq;
    a = make_float4(0.f, 0.f, 0.f, 0.f);
    b = a;
    if (j < L) a = ld4(vb);
    if (j + 1 < L) b = ld4(vb + ld);
  }
  __device__ __forceinline__ void store(uint16_t (*P)[32][kKR], uint16_t (*T)[kHD][kVR]) const {
    int kp, dq;
    tile_slot(threadIdx.x, kp, dq);
    uint2 pa[NP], pb[NP];
    if constexpr (NP == 1) {
      pa[0] = nrfast::hi4(a.x, a.y, a.z, a.w);
      pb[0] = nrfast::hi4(b.x, b.y, b.z, b.w);
    } else {
      nrfast::split4(a.x, a.y, a.z, a.w, pa[0], pa[1], pa[2]);
      nrfast::split4(b.x, b.y, b.z, b.w, pb[0], pb[1], pb[2]);
    }
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      if (P) {
        *reinterpret_cast<uint2*>(&P[q][2 * kp][4 * dq]) = pa[q];
        *reinterpret_cast<uint2*>(&P[q][2 * kp + 1][4 * dq]) = pb[q];
      }
      if (T) {
        *reinterpret_cast<uint32_t*>(&T[q][4 * dq][2 * kp]) = (pa[q].x & 0xffffu) | (pb[q].x << 16);
        *reinterpret_cast<uint32_t*>(&T[q][4 * dq + 1][2 * kp]) = (pa[q].x >> 16) | (pb[q].x & 0xffff0000u);
        *reinterpret_cast<uint32_t*>(&T[q][4 * dq + 2][2 * kp]) = (pa[q].y & 0xffffu) | (pb[q].y << 16);
        *reinterpret_cast<uint32_t*>(&T[q][4 * dq + 3][2 * kp]) = (pa[q].y >> 16) | (pb[q].y & 0xffff0000u);
      }
    }
  }
};

__device__ __forceinline__ float key_add(const AttnArgs& g, int64_t row0, int j, int L) {
  return j >= L ? -INFINITY : (nr_mask_at(g.mask, g.mdt, row0 + j) ? 0.f : kNegMax);
}

// (232 VGPRs: two waves per SIMD.  Bounded to three, 13 spilled and the XFormer step did not move,
// 69.0 vs 69.1 ms, profiles/r04_p_xf_ab.json.)
// W8 (the 501-token user sequence): eight-wave workgroups, threads 0..255 stage K and 256..511 V, so
// each K / V tile is split once per 256 queries instead of per 128 and each thread splits one tensor.
template <int NP, bool DROP, bool PF, bool W8 = false>
__global__ void __launch_bounds__(W8 ? 512 : 256) attn_fwd_mp_kernel(AttnArgs g) {
  __shared__ __attribute__((aligned(16))) uint16_t Kp[NP][32][kKR];
  __shared__ __attribute__((aligned(16))) uint16_t Vt[NP][kHD][kVR];
  __shared__ float kadd[32];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 31, hh = lane >> 5;
  const int nw = blockDim.x >> 6;
  int64_t bid = blockIdx.x;
  const int qc = (int)(bid % g.chunks);
  bid /= g.chunks;
  const int head = (int)(bid % g.heads);
  const int64_t seq = bid / g.heads;
  const int L = g.L;
  const int64_t row0 = seq * L;
  const int q0 = (qc * nw + wave) * 32;
  const bool active = q0 < L;
  const int q = q0 + c;
  const uint32_t dkey = DROP ? attn_key(g, seq, head) : 0u;

  Planes<NP> qp[4];   // B operand of Sᵀ = K Qᵀ: Q[q][32 hh + 8 t + u] / 8 (exact power-of-two scale)
  own_rows<NP>(qp, g.qkv + (row0 + q) * g.ldq + head * kHD + 32 * hh, active && q < L, 0.125f);
  f32x16 o0, o1;
#pragma unroll
  for (int r = 0; r < 16; ++r) o0[r] = o1[r] = 0.f;
  float m = -INFINITY, l = 0.f;
  const int nkb = (L + 31) / 32;
  TileFetch<NP> fk, fv;
  float kadd_n = 0.f;
  const bool kside = threadIdx.x < 256;   // W8: this thread stages K (else V)
  const int64_t wcol = (kside ? g.koff : g.voff) + head * kHD;
  if constexpr (PF) {
    if constexpr (W8) {
      fk.fetch(g.qkv, g.ldq, row0, 0, L, wcol);
    } else {
      fk.fetch(g.qkv, g.ldq, row0, 0, L, g.koff + head * kHD);
      fv.fetch(g.qkv, g.ldq, row0, 0, L, g.voff + head * kHD);
    }
    if (threadIdx.x < 32) kadd_n = key_add(g, row0, threadIdx.x, L);
  }
  for (int kb = 0; kb < nkb; ++kb) {
    __syncthreads();
    if constexpr (PF) {
      if constexpr (W8) {
        if (kside) fk.store(Kp, nullptr);
        else fk.store(nullptr, Vt);
      } else {
        fk.store(Kp, nullptr);
        fv.store(nullptr, Vt);
      }
      if (threadIdx.x < 32) kadd[threadIdx.x] = kadd_n;
      if (kb + 1 < nkb) {
        if constexpr (W8) {
          fk.fetch(g.qkv, g.ldq, row0, (kb + 1) * 32, L, wcol);
        } else {
          fk.fetch(g.qkv, g.ldq, row0, (kb + 1) * 32, L, g.koff + head * kHD);
          fv.fetch(g.qkv, g.ldq, row0, (kb + 1) * 32, L, g.voff + head * kHD);
        }
        if (threadIdx.x < 32) kadd_n = key_add(g, row0, (kb + 1) * 32 + threadIdx.x, L);
      }
    } else {
      stage_planes<NP>(Kp, nullptr, g.qkv, g.ldq, row0, kb * 32, L, g.koff + head * kHD);
      stage_planes<NP>(nullptr, Vt, g.qkv, g.ldq, row0, kb * 32, L, g.voff + head * kHD);
      if (threadIdx.x < 32) kadd[threadIdx.x] = key_add(g, row0, kb * 32 + threadIdx.x, L);
    }
    __syncthreads();
    if (!active) continue;
    f32x16 s;
#pragma unroll
    for (int r = 0; r < 16; ++r) s[r] = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) mfma_x<NP>(s, rowfrag<NP>(Kp, c, hh, t), qp[t]);
    float mx = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      s[r] = s[r] + kadd[crow(r, hh)];
      mx = fmaxf(mx, s[r]);
    }
    mx = xhalf_max(mx);
    const float mn = fmaxf(m, mx);
    const float alpha = __expf(m - mn);
    float ps = 0.f;
    float pe[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      pe[r] = __expf(s[r] - mn);
      ps += pe[r];
    }
    ps = xhalf_sum(ps);
    l = l * alpha + ps;
    m = mn;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      o0[r] *= alpha;
      o1[r] *= alpha;
    }
    if (DROP) {
      uint32_t bits = 0u;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const uint32_t e = (uint32_t)q * (uint32_t)L + (uint32_t)(kb * 32 + crow(r, hh));
        const bool kp = nr_dropout_keep(dkey, e, g.thresh);
        bits |= (kp ? 1u : 0u) << r;
        pe[r] = kp ? pe[r] * g.pscale : 0.f;
      }
      if (g.keep && q < L)   // this lane's half of the (query, key tile) word
        reinterpret_cast<uint16_t*>(g.keep)[2 * keep_word(g, seq, head, q, kb) + hh] = (uint16_t)bits;
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const Planes<NP> pp = planes8<NP>(pe + 8 * t);
      mfma_x<NP>(o0, colfrag<NP>(Vt, c, hh, t), pp);
      mfma_x<NP>(o1, colfrag<NP>(Vt, 32 + c, hh, t), pp);
    }
  }
  if (!active || q >= L) return;
  const float inv = 1.f / l;
  float* op = g.ctx + (row0 + q) * g.ldc + head * kHD;
#pragma unroll
  for (int gq = 0; gq < 4; ++gq) {
    const int d = 8 * gq + 4 * hh;
    st4(op + d, make_float4(o0[4 * gq] * inv, o0[4 * gq + 1] * inv, o0[4 * gq + 2] * inv, o0[4 * gq + 3] * inv));
    st4(op + 32 + d, make_float4(o1[4 * gq] * inv, o1[4 * gq + 1] * inv, o1[4 * gq + 2] * inv, o1[4 * gq + 3] * inv));
  }
  if (hh == 0) {
    float* mp = g.ml + ((row0 + q) * g.heads + head) * 2;
    mp[0] = m;
    mp[1] = inv;
  }
}

// dK, dV (attn_bwd_kv_kernel's products): a wave owns 32 keys, split once; per query tile the Q and
// dctx rows are staged split, row-major (S, dP) and transposed (dV, dK).
// Two waves per SIMD, as attn_bwd_q_mp_kernel: with the own K / V rows held as split planes (96
// VGPRs) the bound spilled 36 and ran slower (profiles/r04_o_xf_ab.json); held as fp32 and split per
// query tile it spills 9 and the XFormer step gains 68.15 -> 67.86 ms (profiles/r04_q_xf_ab.json).
// W8 (the 501-token user sequence): eight-wave workgroups, threads 0..255 stage the Q tile and 256..511
// the dctx tile, so each query tile is split once per 256 keys instead of per 128 (as the forward's W8).
template <int NP, bool DROP, bool PF, bool KB = false, bool DS = false, bool W8 = false>
__global__ void __launch_bounds__(W8 ? 512 : 256) __attribute__((amdgpu_waves_per_eu(2))) attn_bwd_kv_mp_kernel(AttnArgs g) {
  __shared__ __attribute__((aligned(16))) uint16_t Qp[NP][32][kKR];
  __shared__ __attribute__((aligned(16))) uint16_t Op[NP][32][kKR];
  __shared__ __attribute__((aligned(16))) uint16_t Qt[NP][kHD][kVR];
  __shared__ __attribute__((aligned(16))) uint16_t Ot[NP][kHD][kVR];
  __shared__ float qm[32], qi[32], qd[32];
  __shared__ __attribute__((aligned(16))) uint32_t kwd[W8 ? 8 : 4][32];   // per wave: the tile's 32 queries' words of its key tile
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 31, hh = lane >> 5;
  const int nw = blockDim.x >> 6;
  int64_t bid = blockIdx.x;
  const int kc = (int)(bid % g.chunks);
  bid /= g.chunks;
  const int head = (int)(bid % g.heads);
  const int64_t seq = bid / g.heads;
  const int L = g.L;
  const int64_t row0 = seq * L;
  const int k0 = (kc * nw + wave) * 32;
  const bool active = k0 < L;
  const int key = k0 + c;
  const bool own = active && key < L;
  const uint32_t dkey = DROP ? attn_key(g, seq, head) : 0u;

  // the wave's own K / V half-rows kept as fp32 and split per use (planes held for all four steps of
  // both would take 96 VGPRs)
  float kf[32], vf[32];
  {
    const float* kr = g.qkv + (row0 + key) * g.ldq + g.koff + head * kHD + 32 * hh;
    const float* vr = g.qkv + (row0 + key) * g.ldq + g.voff + head * kHD + 32 * hh;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float4 x = own ? ld4(kr + 4 * j) : make_float4(0.f, 0.f, 0.f, 0.f);
      const float4 y = own ? ld4(vr + 4 * j) : make_float4(0.f, 0.f, 0.f, 0.f);
      kf[4 * j] = x.x * 0.125f; kf[4 * j + 1] = x.y * 0.125f; kf[4 * j + 2] = x.z * 0.125f; kf[4 * j + 3] = x.w * 0.125f;
      vf[4 * j] = y.x; vf[4 * j + 1] = y.y; vf[4 * j + 2] = y.z; vf[4 * j + 3] = y.w;
    }
  }
  const float kadd = own ? (nr_mask_at(g.mask, g.mdt, row0 + key) ? 0.f : kNegMax) : -INFINITY;
  // stored keep bits: lane c's key is bit ((c >> 3) << 2 | (c & 3)) + 16 ((c >> 2) & 1) of a query's word
  constexpr bool kbits = DROP && KB;   // KB: g.keep holds the forward's bits (the launcher checks)
  const int kbit = (((c >> 3) << 2) | (c & 3)) + 16 * ((c >> 2) & 1);
  const int kbt = k0 >> 5;   // this wave's key tile
  auto kword = [&](int j) -> uint32_t {   // query j's word of this wave's key tile (0 past L)
    return j < L && active ? g.keep[keep_word(g, seq, head, j, kbt)] : 0u;
  };
  uint32_t kw_n = 0u;
  if (kbits && PF && lane < 32) kw_n = kword(lane);
  f32x16 dk0, dk1, dv0, dv1;
#pragma unroll
  for (int r = 0; r < 16; ++r) dk0[r] = dk1[r] = dv0[r] = dv1[r] = 0.f;
  const int nqb = (L + 31) / 32;
  // a query row's (max, 1/sum, D); past L: exp(s - inf) = 0, no such query
  auto qstats = [&](int j, float& a, float& b, float& d) {
    if (j < L) {
      const float* mp = g.ml + ((row0 + j) * g.heads + head) * 2;
      a = mp[0];
      b = mp[1];
      d = g.Dq[(row0 + j) * g.heads + head];
    } else {
      a = INFINITY;
      b = 0.f;
      d = 0.f;
    }
  };
  TileFetch<NP> fq, fo;
  float qm_n = 0.f, qi_n = 0.f, qd_n = 0.f;
  const bool qside = threadIdx.x < 256;   // W8: this thread stages Q (else dctx)
  const float* wbase = qside ? g.qkv : g.dctx;
  const int64_t wld = qside ? g.ldq : g.ldd;
  if constexpr (PF) {
    if constexpr (W8) {
      fq.fetch(wbase, wld, row0, 0, L, head * kHD);
    } else {
      fq.fetch(g.qkv, g.ldq, row0, 0, L, head * kHD);
      fo.fetch(g.dctx, g.ldd, row0, 0, L, head * kHD);
    }
    if (threadIdx.x < 32) qstats(threadIdx.x, qm_n, qi_n, qd_n);
  }
  for (int qb = 0; qb < nqb; ++qb) {
    __syncthreads();
    if constexpr (PF) {
      if constexpr (W8) {
        if (qside) fq.store(Qp, Qt);
        else fq.store(Op, Ot);
      } else {
        fq.store(Qp, Qt);
        fo.store(Op, Ot);
      }
      if (threadIdx.x < 32) {
        qm[threadIdx.x] = qm_n;
        qi[threadIdx.x] = qi_n;
        qd[threadIdx.x] = qd_n;
      }
      if (kbits && lane < 32) kwd[wave][lane] = kw_n;
      if (qb + 1 < nqb) {
        if constexpr (W8) {
          fq.fetch(wbase, wld, row0, (qb + 1) * 32, L, head * kHD);
        } else {
          fq.fetch(g.qkv, g.ldq, row0, (qb + 1) * 32, L, head * kHD);
          fo.fetch(g.dctx, g.ldd, row0, (qb + 1) * 32, L, head * kHD);
        }
        if (threadIdx.x < 32) qstats((qb + 1) * 32 + threadIdx.x, qm_n, qi_n, qd_n);
        if (kbits && lane < 32) kw_n = kword((qb + 1) * 32 + lane);
      }
    } else {
      stage_planes<NP>(Qp, Qt, g.qkv, g.ldq, row0, qb * 32, L, head * kHD);
      stage_planes<NP>(Op, Ot, g.dctx, g.ldd, row0, qb * 32, L, head * kHD);
      if (threadIdx.x < 32) qstats(qb * 32 + threadIdx.x, qm[threadIdx.x], qi[threadIdx.x], qd[threadIdx.x]);
      if (kbits && lane < 32) kwd[wave][lane] = kword(qb * 32 + lane);
    }
    __syncthreads();
    if (!active) continue;
    // this lane's keep bits of the 16 queries crow(r, hh) (four runs of four consecutive words): bit r
    uint32_t kmask = 0u;
    if constexpr (kbits) {
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const uint4 w4 = *reinterpret_cast<const uint4*>(&kwd[wave][8 * g4 + 4 * hh]);
        kmask |= (((w4.x >> kbit) & 1u) | (((w4.y >> kbit) & 1u) << 1) | (((w4.z >> kbit) & 1u) << 2) |
                  (((w4.w >> kbit) & 1u) << 3)) << (4 * g4);
        asm volatile("" : "+v"(kmask));   // one run's four words live at a time
      }
    }
    f32x16 s, dp;
#pragma unroll
    for (int r = 0; r < 16; ++r) s[r] = dp[r] = 0.f;
#pragma unroll
    for (int j = 0; j < 32; ++j) asm volatile("" : "+v"(kf[j]), "+v"(vf[j]));   // split per tile, not hoisted
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      mfma_x<NP>(s, rowfrag<NP>(Qp, c, hh, t), planes8<NP>(kf + 8 * t));
      mfma_x<NP>(dp, rowfrag<NP>(Op, c, hh, t), planes8<NP>(vf + 8 * t));
    }
    // S rows = queries crow(r, hh) of the tile, column = this lane's key
    float pd[16], ds[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int qr = crow(r, hh);
      const float pr = __expf(s[r] + kadd - qm[qr]) * qi[qr];
      float d = dp[r];
      float pdr = pr;
      if (DROP) {
        bool kp;
        if constexpr (kbits) {
          kp = (kmask >> r) & 1u;
        } else {
          const uint32_t e = (uint32_t)(qb * 32 + qr) * (uint32_t)L + (uint32_t)key;
          kp = nr_dropout_keep(dkey, e, g.thresh);
        }
        d = kp ? d * g.pscale : 0.f;
        pdr = kp ? pr * g.pscale : 0.f;
      }
      pd[r] = pdr;
      ds[r] = pr * (d - qd[qr]);
    }
    if constexpr (DS) {   // one 128 B row (query) per half-wave and r, unconditional: keys past L
      // and the padding queries L .. 32 nkb - 1 store 0 (p = 0 there)
      float* dsp = g.dsb + (((seq * g.heads + head) * (int64_t)g.nkb + kbt) * g.nkb + qb) * 1024 + c;
#pragma unroll
      for (int r = 0; r < 16; ++r) dsp[crow(r, hh) * 32] = ds[r];
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const Planes<NP> pp = planes8<NP>(pd + 8 * t), sp = planes8<NP>(ds + 8 * t);
      mfma_x<NP>(dv0, colfrag<NP>(Ot, c, hh, t), pp);
      mfma_x<NP>(dv1, colfrag<NP>(Ot, 32 + c, hh, t), pp);
      mfma_x<NP>(dk0, colfrag<NP>(Qt, c, hh, t), sp);
      mfma_x<NP>(dk1, colfrag<NP>(Qt, 32 + c, hh, t), sp);
    }
  }
  if (!own) return;
  float* kp = g.dqkv + (row0 + key) * g.lddq + g.koff + head * kHD;
  float* vp = g.dqkv + (row0 + key) * g.lddq + g.voff + head * kHD;
#pragma unroll
  for (int gq = 0; gq < 4; ++gq) {
    const int d = 8 * gq + 4 * hh;
    st4(kp + d, make_float4(dk0[4 * gq] * 0.125f, dk0[4 * gq + 1] * 0.125f, dk0[4 * gq + 2] * 0.125f,
                            dk0[4 * gq + 3] * 0.125f));
    st4(kp + 32 + d, make_float4(dk1[4 * gq] * 0.125f, dk1[4 * gq + 1] * 0.125f, dk1[4 * gq + 2] * 0.125f,
                                 dk1[4 * gq + 3] * 0.125f));
    st4(vp + d, make_float4(dv0[4 * gq], dv0[4 * gq + 1], dv0[4 * gq + 2], dv0[4 * gq + 3]));
    st4(vp + 32 + d, make_float4(dv1[4 * gq], dv1[4 * gq + 1], dv1[4 * gq + 2], dv1[4 * gq + 3]));
  }
}

// dQ (attn_bwd_q_kernel's products): a wave owns 32 queries (Q and dctx split once); per key tile
// K and V staged split row-major (S, dP) and K transposed (dQ = dS K).
// Two waves per SIMD: unbounded, the bf16x6 prefetching form took 270 VGPRs -- one wave per SIMD,
// its softmax / dS arithmetic never overlapping another wave's MFMAs; at <= 256 it fits without
// spills: XFormer step 71.5 -> 69.9 ms on one box (profiles/r04_o_xf_ab.json).
template <int NP, bool DROP, bool PF, bool KB = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) attn_bwd_q_mp_kernel(AttnArgs g) {
  __shared__ __attribute__((aligned(16))) uint16_t Kp[NP][32][kKR];
  __shared__ __attribute__((aligned(16))) uint16_t Vp[NP][32][kKR];
  __shared__ __attribute__((aligned(16))) uint16_t Kt[NP][kHD][kVR];
  __shared__ float kadd[32];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 31, hh = lane >> 5;
  const int nw = blockDim.x >> 6;
  int64_t bid = blockIdx.x;
  const int qc = (int)(bid % g.chunks);
  bid /= g.chunks;
  const int head = (int)(bid % g.heads);
  const int64_t seq = bid / g.heads;
  const int L = g.L;
  const int64_t row0 = seq * L;
  const int q0 = (qc * nw + wave) * 32;
  const bool active = q0 < L;
  const int q = q0 + c;
  const bool own = active && q < L;
  const uint32_t dkey = DROP ? attn_key(g, seq, head) : 0u;

  Planes<NP> qp4[4], dp4[4];
  own_rows<NP>(qp4, g.qkv + (row0 + q) * g.ldq + head * kHD + 32 * hh, own, 0.125f);
  own_rows<NP>(dp4, g.dctx + (row0 + q) * g.ldd + head * kHD + 32 * hh, own, 1.f);
  float mq = INFINITY, iq = 0.f, dq = 0.f;
  if (own) {
    const float* mp = g.ml + ((row0 + q) * g.heads + head) * 2;
    mq = mp[0];
    iq = mp[1];
    dq = g.Dq[(row0 + q) * g.heads + head];
  }
  f32x16 a0, a1;
#pragma unroll
  for (int r = 0; r < 16; ++r) a0[r] = a1[r] = 0.f;
  const int nkb = (L + 31) / 32;
  // stored keep bits: this lane's half of its query's word of each key tile, loaded a tile ahead
  constexpr bool kbits = DROP && KB;   // KB: g.keep holds the forward's bits (the launcher checks)
  auto kword = [&](int kb) -> uint32_t { return own ? g.keep[keep_word(g, seq, head, q, kb)] >> (16 * hh) : 0u; };
  uint32_t kw_c = kbits ? kword(0) : 0u;
  TileFetch<NP> fk, fv;
  float kadd_n = 0.f;
  if constexpr (PF) {
    fk.fetch(g.qkv, g.ldq, row0, 0, L, g.koff + head * kHD);
    fv.fetch(g.qkv, g.ldq, row0, 0, L, g.voff + head * kHD);
    if (threadIdx.x < 32) kadd_n = key_add(g, row0, threadIdx.x, L);
  }
  for (int kb = 0; kb < nkb; ++kb) {
    const uint32_t kw = kw_c;
    if (kbits && kb + 1 < nkb) kw_c = kword(kb + 1);
    __syncthreads();
    if constexpr (PF) {
      fk.store(Kp, Kt);
      fv.store(Vp, nullptr);
      if (threadIdx.x < 32) kadd[threadIdx.x] = kadd_n;
      if (kb + 1 < nkb) {
        fk.fetch(g.qkv, g.ldq, row0, (kb + 1) * 32, L, g.koff + head * kHD);
        fv.fetch(g.qkv, g.ldq, row0, (kb + 1) * 32, L, g.voff + head * kHD);
        if (threadIdx.x < 32) kadd_n = key_add(g, row0, (kb + 1) * 32 + threadIdx.x, L);
      }
    } else {
      stage_planes<NP>(Kp, Kt, g.qkv, g.ldq, row0, kb * 32, L, g.koff + head * kHD);
      stage_planes<NP>(Vp, nullptr, g.qkv, g.ldq, row0, kb * 32, L, g.voff + head * kHD);
      if (threadIdx.x < 32) kadd[threadIdx.x] = key_add(g, row0, kb * 32 + threadIdx.x, L);
    }
    __syncthreads();
    if (!active) continue;
    f32x16 s, dp;
#pragma unroll
    for (int r = 0; r < 16; ++r) s[r] = dp[r] = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      mfma_x<NP>(s, rowfrag<NP>(Kp, c, hh, t), qp4[t]);
      mfma_x<NP>(dp, rowfrag<NP>(Vp, c, hh, t), dp4[t]);
    }
    float ds[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int kr = crow(r, hh);
      const float pr = __expf(s[r] + kadd[kr] - mq) * iq;
      float d = dp[r];
      if (DROP) {
        bool kp;
        if constexpr (kbits) {
          kp = (kw >> r) & 1u;
        } else {
          const uint32_t e = (uint32_t)q * (uint32_t)L + (uint32_t)(kb * 32 + kr);
          kp = nr_dropout_keep(dkey, e, g.thresh);
        }
        d = kp ? d * g.pscale : 0.f;
      }
      ds[r] = pr * (d - dq);
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const Planes<NP> sp = planes8<NP>(ds + 8 * t);
      mfma_x<NP>(a0, colfrag<NP>(Kt, c, hh, t), sp);
      mfma_x<NP>(a1, colfrag<NP>(Kt, 32 + c, hh, t), sp);
    }
  }
  if (!own) return;
  float* op = g.dqkv + (row0 + q) * g.lddq + head * kHD;
#pragma unroll
  for (int gq = 0; gq < 4; ++gq) {
    const int d = 8 * gq + 4 * hh;
    st4(op + d, make_float4(a0[4 * gq] * 0.125f, a0[4 * gq + 1] * 0.125f, a0[4 * gq + 2] * 0.125f,
                            a0[4 * gq + 3] * 0.125f));
    st4(op + 32 + d, make_float4(a1[4 * gq] * 0.125f, a1[4 * gq + 1] * 0.125f, a1[4 * gq + 2] * 0.125f,
                                 a1[4 * gq + 3] * 0.125f));
  }
}

// dQ = dS K from the dS tiles attn_bwd_kv_mp_kernel<..., DS = true> stored (four-wave launches, the
// 501-token user sequence): a wave owns 32 queries; per key tile only K is staged (transposed) and
// lane (c, h) loads its query's 16 dS values of the tile (four float4, a tile ahead) -- no S, P, dP
// recompute, no dropout hash, no Q / dctx planes in registers.
template <int NP>
__global__ void __launch_bounds__(256) attn_bwd_q_ds_kernel(AttnArgs g) {
  __shared__ __attribute__((aligned(16))) uint16_t Kt[NP][kHD][kVR];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 31, hh = lane >> 5;
  int64_t bid = blockIdx.x;
  const int qc = (int)(bid % g.chunks);
  bid /= g.chunks;
  const int head = (int)(bid % g.heads);
  const int64_t seq = bid / g.heads;
  const int L = g.L;
  const int64_t row0 = seq * L;
  const int q0 = (qc * 4 + wave) * 32;
  const bool active = q0 < L;
  const int q = q0 + c;
  const bool own = active && q < L;
  const int nkb = (L + 31) / 32;
  // slot r = 4 j + u of key tile kb: key kb * 32 + crow(r, h) = 8 j + 4 h + u
  const float* dsp = g.dsb + ((seq * g.heads + head) * (int64_t)g.nkb * g.nkb * 32 + q) * 32 + 4 * hh;
  auto load = [&](int kb, float (&d)[16]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float4 x = own ? ld4(dsp + (int64_t)kb * g.nkb * 1024 + 8 * j) : make_float4(0.f, 0.f, 0.f, 0.f);
      d[4 * j] = x.x; d[4 * j + 1] = x.y; d[4 * j + 2] = x.z; d[4 * j + 3] = x.w;
    }
  };
  f32x16 a0, a1;
#pragma unroll
  for (int r = 0; r < 16; ++r) a0[r] = a1[r] = 0.f;
  TileFetch<NP> fk;
  fk.fetch(g.qkv, g.ldq, row0, 0, L, g.koff + head * kHD);
  float dn[16];
  load(0, dn);
  for (int kb = 0; kb < nkb; ++kb) {
    float ds[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) ds[r] = dn[r];
    __syncthreads();
    fk.store(nullptr, Kt);
    if (kb + 1 < nkb) {
      fk.fetch(g.qkv, g.ldq, row0, (kb + 1) * 32, L, g.koff + head * kHD);
      load(kb + 1, dn);
    }
    __syncthreads();
    if (!active) continue;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const Planes<NP> sp = planes8<NP>(ds + 8 * t);
      mfma_x<NP>(a0, colfrag<NP>(Kt, c, hh, t), sp);
      mfma_x<NP>(a1, colfrag<NP>(Kt, 32 + c, hh, t), sp);
    }
  }
  if (!own) return;
  float* op = g.dqkv + (row0 + q) * g.lddq + head * kHD;
#pragma unroll
  for (int gq = 0; gq < 4; ++gq) {
    const int d = 8 * gq + 4 * hh;
    st4(op + d, make_float4(a0[4 * gq] * 0.125f, a0[4 * gq + 1] * 0.125f, a0[4 * gq + 2] * 0.125f,
                            a0[4 * gq + 3] * 0.125f));
    st4(op + 32 + d, make_float4(a1[4 * gq] * 0.125f, a1[4 * gq + 1] * 0.125f, a1[4 * gq + 2] * 0.125f,
                                 a1[4 * gq + 3] * 0.125f));
  }
}

__global__ void __launch_bounds__(256) tanh_bwd_kernel(const float* y, int64_t ldy, const float* dy, int64_t lddy,
                                                       int64_t rows, int cols, float* dx, int64_t lddx) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * cols) return;
  const int64_t r = i / cols;
  const int c = (int)(i - r * cols);
  const float v = y[r * ldy + c];
  dx[r * lddx + c] = dy[r * lddy + c] * (1.f - v * v);
}

bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

int attn_setup(AttnArgs& g, const float* qkv, int64_t ldq, int64_t koff, int64_t voff, const void* mask,
               int32_t mdt, int64_t nseq, int32_t L, int32_t heads, float p, uint64_t seed, uint64_t offset,
               const uint64_t* rng, float* ml) {
  if (nseq < 0 || L <= 0 || heads <= 0) return NR_EINVAL(0);
  if (!qkv || !mask || !ml) return NR_EINVAL(1);
  if (!al16(qkv) || (ldq & 3) || (koff & 3) || (voff & 3)) return NR_EINVAL(2);
  if (p < 0.f || p >= 1.f) return NR_EINVAL(3);
  g.qkv = qkv; g.ldq = ldq; g.koff = koff; g.voff = voff; g.mask = mask; g.mdt = mdt;
  g.nseq = nseq; g.L = L; g.heads = heads;
  g.p = p; g.pscale = p > 0.f ? 1.f / (1.f - p) : 1.f; g.thresh = nr_dropout_threshold(p);
  g.key = nr_dropout_key(seed, offset); g.rng = rng; g.offset = offset; g.ml = ml;
  return NR_OK;
}

bool prec_ok(int32_t prec) { return prec == NR_GEMM_F32 || prec == NR_GEMM_BF16X6 || prec == NR_GEMM_BF16; }

// waves per workgroup: enough to cover L with 32-row waves, at most 4
int attn_waves(int L) {
  const int w = (L + 31) / 32;
  return w < 4 ? w : 4;
}

}  // namespace

// ==================================================================================== C ABI

extern "C" int nr_bert_embed_fwd(const float* word, int64_t V, const float* pos, int64_t P, const float* type0,
                                 const int64_t* ids, int64_t nseq, int32_t L, int32_t H, const float* gamma,
                                 const float* beta, float eps, float p_drop, uint64_t seed, uint64_t offset,
                                 const uint64_t* rng, float* out, int64_t ldo, float* stats, int32_t* status,
                                 hipStream_t stream) {
  if (nseq < 0 || L <= 0 || H <= 0 || (H & 3) || H > 1024) return NR_EINVAL(0);
  if (L > P) return NR_EINVAL(3);
  if (!word || !pos || !type0 || !ids || !gamma || !beta || !out || !stats) return NR_EINVAL(1);
  if (!al16(word) || !al16(pos) || !al16(type0) || !al16(out) || (ldo & 3)) return NR_EINVAL(2);
  LnArgs g{};
  g.word = word; g.V = V; g.pos = pos; g.type0 = type0; g.ids = ids; g.L = L;
  g.T = nseq * L; g.H = H; g.gamma = gamma; g.beta = beta; g.eps = eps;
  set_drop(g, p_drop, seed, offset, rng);
  g.out = out; g.ldo = ldo; g.stats = stats; g.status = status;
  return launch_ln<true, false>(g, stream);
}

extern "C" int nr_bert_embed_bwd(const float* word, int64_t V, const float* pos, const float* type0,
                                 const int64_t* ids, int64_t nseq, int32_t L, int32_t H, const float* gamma,
                                 float p_drop, uint64_t seed, uint64_t offset, const uint64_t* rng,
                                 const float* stats, const float* dout, int64_t ldd, float* ds, int64_t ldds,
                                 float* dgamma, float* dbeta, hipStream_t stream) {
  if (nseq < 0 || L <= 0 || H <= 0 || (H & 3) || H > 1024) return NR_EINVAL(0);
  if (!word || !pos || !type0 || !ids || !gamma || !stats || !dout || !ds || !dgamma || !dbeta) return NR_EINVAL(1);
  if (!al16(dout) || !al16(ds) || (ldd & 3) || (ldds & 3)) return NR_EINVAL(2);
  LnArgs g{};
  g.word = word; g.V = V; g.pos = pos; g.type0 = type0; g.ids = ids; g.L = L;
  g.T = nseq * L; g.H = H; g.gamma = gamma;
  set_drop(g, p_drop, seed, offset, rng);
  g.stats = const_cast<float*>(stats); g.dout = dout; g.ldd = ldd; g.ds = ds; g.ldds = ldds; g.dgamma = dgamma; g.dbeta = dbeta;
  return launch_ln<true, true>(g, stream);
}

extern "C" int nr_bert_add_ln_fwd(const float* x, int64_t ldx, const float* res, int64_t ldr, int64_t T, int32_t H,
                                  const float* gamma, const float* beta, float eps, float p_drop, uint64_t seed,
                                  uint64_t offset, const uint64_t* rng, float* out, int64_t ldo, float* stats,
                                  hipStream_t stream) {
  if (T < 0 || H <= 0 || (H & 3) || H > 1024) return NR_EINVAL(0);
  if (!x || !res || !gamma || !beta || !out || !stats) return NR_EINVAL(1);
  if (!al16(x) || !al16(res) || !al16(out) || (ldx & 3) || (ldr & 3) || (ldo & 3)) return NR_EINVAL(2);
  LnArgs g{};
  g.x = x; g.ldx = ldx; g.res = res; g.ldr = ldr; g.T = T; g.H = H; g.gamma = gamma; g.beta = beta; g.eps = eps;
  set_drop(g, p_drop, seed, offset, rng);
  g.out = out; g.ldo = ldo; g.stats = stats;
  return launch_ln<false, false>(g, stream);
}

extern "C" int nr_bert_add_ln_bwd(const float* x, int64_t ldx, const float* res, int64_t ldr, int64_t T, int32_t H,
                                  const float* gamma, float p_drop, uint64_t seed, uint64_t offset,
                                  const uint64_t* rng, const float* stats, const float* dout, int64_t ldd,
                                  float* dres, int64_t lddr, float* dx, int64_t lddx, float* dgamma, float* dbeta,
                                  hipStream_t stream) {
  if (T < 0 || H <= 0 || (H & 3) || H > 1024) return NR_EINVAL(0);
  if (!x || !res || !gamma || !stats || !dout || !dres || !dx || !dgamma || !dbeta) return NR_EINVAL(1);
  if (!al16(x) || !al16(res) || !al16(dout) || !al16(dres) || !al16(dx) || ((ldx | ldr | ldd | lddr | lddx) & 3))
    return NR_EINVAL(2);
  LnArgs g{};
  g.x = x; g.ldx = ldx; g.res = res; g.ldr = ldr; g.T = T; g.H = H; g.gamma = gamma;
  set_drop(g, p_drop, seed, offset, rng);
  g.stats = const_cast<float*>(stats); g.dout = dout; g.ldd = ldd; g.ds = dres; g.ldds = lddr; g.dx = dx; g.lddx = lddx;
  g.dgamma = dgamma; g.dbeta = dbeta;
  return launch_ln<false, true>(g, stream);
}

extern "C" int64_t nr_bert_attn_keep_words(int64_t nseq, int32_t L, int32_t heads) {
  if (nseq < 0 || L <= 0 || heads <= 0) return 0;
  return nseq * heads * (int64_t)L * ((L + 31) / 32);
}

extern "C" int nr_bert_attn_fwd(const float* qkv, int64_t ldq, int64_t koff, int64_t voff, const void* mask,
                                int32_t mask_dtype, int64_t nseq, int32_t L, int32_t heads, float p_drop,
                                uint64_t seed, uint64_t offset, const uint64_t* rng, float* ctx, int64_t ldc,
                                float* ml, uint32_t* keep, int32_t prec, hipStream_t stream) {
  AttnArgs g{};
  int rc = attn_setup(g, qkv, ldq, koff, voff, mask, mask_dtype, nseq, L, heads, p_drop, seed, offset, rng, ml);
  if (rc) return rc;
  if (!ctx || !al16(ctx) || (ldc & 3)) return NR_EINVAL(4);
  if (!prec_ok(prec)) return NR_EINVAL(6);
  if (keep && prec == NR_GEMM_F32) return NR_EINVAL(7);   // the f32 forward does not store keep bits
  if (nseq == 0) return NR_OK;
  g.ctx = ctx; g.ldc = ldc;
  g.keep = p_drop > 0.f ? keep : nullptr; g.nkb = (L + 31) / 32;
  // four-wave sequences (L > 96) with the MFMA arithmetic run as eight-wave workgroups (W8)
  const int nw = attn_waves(L) == 4 && prec != NR_GEMM_F32 ? 8 : attn_waves(L);
  g.chunks = (L + 32 * nw - 1) / (32 * nw);
  const dim3 grid((unsigned)(nseq * heads * g.chunks)), block(64 * nw);
  const bool drop = p_drop > 0.f;
#define NR_FWD(KER) hipLaunchKernelGGL(KER, grid, block, 0, stream, g)
  if (prec == NR_GEMM_F32) {
    if (drop) NR_FWD(attn_fwd_kernel<true>);
    else NR_FWD(attn_fwd_kernel<false>);
  } else if (nw == 8) {
    if (prec == NR_GEMM_BF16) {
      if (drop) NR_FWD((attn_fwd_mp_kernel<1, true, true, true>));
      else NR_FWD((attn_fwd_mp_kernel<1, false, true, true>));
    } else {
      if (drop) NR_FWD((attn_fwd_mp_kernel<3, true, true, true>));
      else NR_FWD((attn_fwd_mp_kernel<3, false, true, true>));
    }
  } else if (prec == NR_GEMM_BF16) {
    if (drop) NR_FWD((attn_fwd_mp_kernel<1, true, false>));
    else NR_FWD((attn_fwd_mp_kernel<1, false, false>));
  } else {
    if (drop) NR_FWD((attn_fwd_mp_kernel<3, true, false>));
    else NR_FWD((attn_fwd_mp_kernel<3, false, false>));
  }
#undef NR_FWD
  NR_LAUNCH_CHECK();
  return NR_OK;
}

namespace {
// floats of the workspace ahead of the dS tiles: D, rounded up to 16 B
int64_t attn_dq_floats(int64_t nseq, int32_t L, int32_t heads) { return (nseq * (int64_t)L * heads + 3) & ~(int64_t)3; }
}  // namespace

extern "C" int64_t nr_bert_attn_bwd_workspace(int64_t nseq, int32_t L, int32_t heads) {
  if (nseq < 0 || L <= 0 || heads <= 0) return 0;
  int64_t f = attn_dq_floats(nseq, L, heads);
  const int64_t nkb = (L + 31) / 32;
  if (attn_waves(L) == 4) f += nseq * heads * nkb * nkb * 1024;   // dS tiles
  return f * (int64_t)sizeof(float);
}

extern "C" int nr_bert_attn_bwd(const float* qkv, int64_t ldq, int64_t koff, int64_t voff, const void* mask,
                                int32_t mask_dtype, int64_t nseq, int32_t L, int32_t heads, float p_drop,
                                uint64_t seed, uint64_t offset, const uint64_t* rng, const float* ctx, int64_t ldc,
                                const float* ml, const uint32_t* keep, const float* dctx, int64_t ldd, float* work,
                                float* dqkv, int64_t lddq, int32_t prec, hipStream_t stream) {
  AttnArgs g{};
  int rc = attn_setup(g, qkv, ldq, koff, voff, mask, mask_dtype, nseq, L, heads, p_drop, seed, offset, rng,
                      const_cast<float*>(ml));
  if (rc) return rc;
  if (!ctx || !dctx || !work || !dqkv) return NR_EINVAL(4);
  if (!al16(ctx) || !al16(dctx) || !al16(dqkv) || !al16(work) || ((ldc | ldd | lddq) & 3)) return NR_EINVAL(5);
  if (!prec_ok(prec)) return NR_EINVAL(6);
  if (nseq == 0) return NR_OK;
  const int64_t T = nseq * L;
  g.dsb = work + attn_dq_floats(nseq, L, heads);
  hipLaunchKernelGGL(attn_dsum_kernel, dim3((unsigned)((T * heads * (kHD / 4) + 255) / 256)), dim3(256), 0, stream, dctx,
                     ldd, ctx, ldc, T, heads, work);
  NR_LAUNCH_CHECK();
  g.dctx = dctx; g.ldd = ldd; g.Dq = work; g.dqkv = dqkv; g.lddq = lddq;
  // the f32 kernels re-hash (their forward stored no bits: the same masks either way)
  g.keep = p_drop > 0.f && prec != NR_GEMM_F32 ? const_cast<uint32_t*>(keep) : nullptr;
  g.nkb = (L + 31) / 32;
  const int nw = attn_waves(L);
  g.chunks = (L + 32 * nw - 1) / (32 * nw);
  const dim3 grid((unsigned)(nseq * heads * g.chunks)), block(64 * nw);
  const bool drop = p_drop > 0.f;
  // the dK/dV pass of four-wave sequences with the MFMA arithmetic runs as eight-wave workgroups (W8)
  const bool w8 = nw == 4 && prec != NR_GEMM_F32 && kNrAttnBwdW8;   // (the f32 kernels are 256-thread)
  AttnArgs gkv = g;
  gkv.chunks = w8 ? (L + 255) / 256 : g.chunks;
  const dim3 gridkv((unsigned)(nseq * heads * gkv.chunks)), blockkv(w8 ? 512 : 64 * nw);
#define NR_BWD(KV, Q)                                          \
  do {                                                         \
    hipLaunchKernelGGL(KV, gridkv, blockkv, 0, stream, gkv);   \
    hipLaunchKernelGGL(Q, grid, block, 0, stream, g);          \
  } while (0)
  const bool kb = drop && g.keep != nullptr;
  if (prec == NR_GEMM_F32) {
    if (drop) NR_BWD(attn_bwd_kv_kernel<true>, attn_bwd_q_kernel<true>);
    else NR_BWD(attn_bwd_kv_kernel<false>, attn_bwd_q_kernel<false>);
  } else if (kb && w8) {   // the forward's keep bits instead of the per-element hash
    if (prec == NR_GEMM_BF16) NR_BWD((attn_bwd_kv_mp_kernel<1, true, true, true, true, true>), attn_bwd_q_ds_kernel<1>);
    else NR_BWD((attn_bwd_kv_mp_kernel<3, true, true, true, true, true>), attn_bwd_q_ds_kernel<3>);
  } else if (kb && nw == 4) {
    if (prec == NR_GEMM_BF16) NR_BWD((attn_bwd_kv_mp_kernel<1, true, true, true, true>), attn_bwd_q_ds_kernel<1>);
    else NR_BWD((attn_bwd_kv_mp_kernel<3, true, true, true, true>), attn_bwd_q_ds_kernel<3>);
  } else if (kb) {
    if (prec == NR_GEMM_BF16) NR_BWD((attn_bwd_kv_mp_kernel<1, true, false, true>), (attn_bwd_q_mp_kernel<1, true, false, true>));
    else NR_BWD((attn_bwd_kv_mp_kernel<3, true, false, true>), (attn_bwd_q_mp_kernel<3, true, false, true>));
  } else if (w8) {
    if (prec == NR_GEMM_BF16) {
      if (drop) NR_BWD((attn_bwd_kv_mp_kernel<1, true, true, false, true, true>), attn_bwd_q_ds_kernel<1>);
      else NR_BWD((attn_bwd_kv_mp_kernel<1, false, true, false, true, true>), attn_bwd_q_ds_kernel<1>);
    } else {
      if (drop) NR_BWD((attn_bwd_kv_mp_kernel<3, true, true, false, true, true>), attn_bwd_q_ds_kernel<3>);
      else NR_BWD((attn_bwd_kv_mp_kernel<3, false, true, false, true, true>), attn_bwd_q_ds_kernel<3>);
    }
  } else if (nw == 4) {
    if (prec == NR_GEMM_BF16) {
      if (drop) NR_BWD((attn_bwd_kv_mp_kernel<1, true, true, false, true>), attn_bwd_q_ds_kernel<1>);
      else NR_BWD((attn_bwd_kv_mp_kernel<1, false, true, false, true>), attn_bwd_q_ds_kernel<1>);
    } else {
      if (drop) NR_BWD((attn_bwd_kv_mp_kernel<3, true, true, false, true>), attn_bwd_q_ds_kernel<3>);
      else NR_BWD((attn_bwd_kv_mp_kernel<3, false, true, false, true>), attn_bwd_q_ds_kernel<3>);
    }
  } else if (prec == NR_GEMM_BF16) {
    if (drop) NR_BWD((attn_bwd_kv_mp_kernel<1, true, false>), (attn_bwd_q_mp_kernel<1, true, false>));
    else NR_BWD((attn_bwd_kv_mp_kernel<1, false, false>), (attn_bwd_q_mp_kernel<1, false, false>));
  } else {
    if (drop) NR_BWD((attn_bwd_kv_mp_kernel<3, true, false>), (attn_bwd_q_mp_kernel<3, true, false>));
    else NR_BWD((attn_bwd_kv_mp_kernel<3, false, false>), (attn_bwd_q_mp_kernel<3, false, false>));
  }
#undef NR_BWD
  NR_LAUNCH_CHECK();
  return NR_OK;
}

extern "C" int nr_tanh_bwd(const float* y, int64_t ldy, const float* dy, int64_t lddy, int64_t rows, int32_t cols,
                           float* dx, int64_t lddx, hipStream_t stream) {
  if (rows < 0 || cols < 0) return NR_EINVAL(0);
  if (!y || !dy || !dx) return NR_EINVAL(1);
  if (rows * cols == 0) return NR_OK;
  hipLaunchKernelGGL(tanh_bwd_kernel, dim3((unsigned)((rows * cols + 255) / 256)), dim3(256), 0, stream, y, ldy, dy,
                     lddy, rows, cols, dx, lddx);
  NR_LAUNCH_CHECK();
  return NR_OK;
}
