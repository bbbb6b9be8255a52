// Fused MHA news encoder tail, one workgroup per title (L <= 32 tokens):
//
//   per head h:  S = Kp_h Kp_hᵀ · scale          (Q = K = keyProject(x), Attention.py:125-126)
//                P = XSoftmax(S, m_i m_j)         (Attention.py:56-80, pairwise mask :33-53)
//                O_h = P Vp_h                     (heads concatenated, no output projection)
//   Z = Dropout(LayerNorm(O));  news = Σ_l XSoftmax(q·Z_l / sqrt(H))_l Z_l     (MHA.py:37-38)
//
// The attention runs on the f32 matrix cores (v_mfma_f32_32x32x2_f32, exact fp32) with the
// title padded to a 32x32 tile, one wave per head:
//   * S needs no LDS: lane (c, half) holds its own key row's half (K[c][half*DK/2 ..]) and
//     feeds it as BOTH operands (A = K, B = Kᵀ use the same register).
//   * S is symmetric, so the accumulator (column c on the lane) is also ROW c of S: the row
//     softmax is 16 in-register values + one cross-half exchange, and P lands in the layout
//     an A operand needs for the next product — O = P V takes P straight from registers with
//     the k index permuted to the accumulator's row order (crow below).
// O is staged in LDS [L x H], then LayerNorm / dropout (stateless counter RNG) / pooling run
// on it in the same workgroup: the [T, H] attention output never touches HBM.
//
// The backward recomputes S, P, O from the projections, runs the pooling / dropout / LN
// backward in LDS, then per head dPᵀ = V dOᵀ, dS = P∘(dP − rowsum), the symmetric
// dKp = scale (dS + dSᵀ) Kp and dVp = Pᵀ dO, with the transposes through a per-wave 32x33 LDS
// tile, and accumulates the projection-bias gradient (column sums of dY) in the epilogue.
#include "common.h"
#include "../../include/newsrec_hip.h"
#include <stdlib.h>

#include "mfma_planes.h"   // Planes / mfma16 / crow / wave_lds_fence

namespace {

struct MPArgs {
  const float* y; int64_t ldy;        // [T][heads*dk + heads*dv] projections
  const int64_t* yrows;               // optional: projection row of token t
  const void* mask; int mask_dt;      // [nseq][L]
  int64_t nseq; int L; int heads;
  float scale_attn, scale_pool;
  const float* gamma; const float* beta; float eps;
  float p_drop; uint64_t seed; uint64_t offset;
  uint32_t dkey, dthresh;                  // dropout key / threshold derived on the host
  const uint64_t* rng;                     // device (seed, offset base): key derived in the kernel
  const float* q;                     // [H] query_words
  float* news; int64_t ldn;           // fwd out / bwd: dnews in (const)
  float* zout; int64_t ldz;           // fwd: optional token output Z
  float* stats; float* probs;         // [T][2], [T]
  const float* dz; int64_t lddz;      // bwd: optional grad of Z
  float* dy; int64_t lddy;            // bwd: [T][heads*dk + heads*dv]
  // bwd, optional: the CSR offsets of the distinct rows' gradient-carrying tokens (nr_unique_rows):
  // a token alone in its row's segment writes its dy row straight to row dyu_row0 + yrows[t] of dy
  // (the per-distinct-row sum the segment sum would form), masked tokens write nothing
  const int32_t* seg_off; int64_t dyu_row0;
  uint32_t* dsto;                     // split bwd with seg_off: per-token dy byte offsets (LN pass writes)
  float* dbias; float* dq; float* dgamma; float* dbeta;
  float* o; int64_t ldo;              // fwd: optional saved attention output O (pre-LN); bwd: its input
  float* dob; int64_t lddob;          // split bwd: dO rows (kernel 1 writes, kernel 2 reads)
  int rows_per_wave;                  // staged row indices per wave (split bwd kernel 2) or per block
  int np;                             // attention products: 0 = f32 MFMA, 3 = bf16x6, 1 = bf16
  float* ws; int ws_copies; int64_t ws_ld;   // split bwd: parameter-gradient copies (see nr_mha_pool_bwd)
};

// Parameter-gradient partials of the split backward: workgroup b adds into copy b % ws_copies of
// [dgamma | dbeta | dq | dbias] instead of the single vectors -- 1,760 titles' atomics on the same
// 2,304 addresses serialise at L2 (measured: ≈ 38 us of the backward); copies_reduce_kernel then
// folds the copies into the outputs.
__device__ __forceinline__ float* grad_slot(const MPArgs& g, int64_t col_in_ws) {
  return g.ws + (int64_t)(blockIdx.x % g.ws_copies) * g.ws_ld + col_in_ws;
}

// Projection rows of the workgroup's title are staged once per title as 32-bit BYTE offsets
// from y (yrows[token] * ldy * 4, or the token's own row) in the first 32 words of the dynamic
// LDS (per wave in the split backward), so the per-head K/V loads never wait on an index load
// and address as 64-bit SGPR base + 32-bit VGPR offset (one VGPR per address, not two).
// Requires (rows of y) * ldy * 4 < 2^32.
__device__ __forceinline__ uint32_t yrow_off(const MPArgs& g, int l) {
  extern __shared__ uint32_t nr_mp_rows[];
  const int base = g.rows_per_wave ? (int)(threadIdx.x >> 6) * 32 : 0;
  return nr_mp_rows[base + l];
}

__device__ __forceinline__ float ld_off(const float* base, uint32_t byte_off) {
  return *reinterpret_cast<const float*>(reinterpret_cast<const char*>(base) + byte_off);
}

__device__ __forceinline__ void st_off(float* base, uint32_t byte_off, float v) {
  *reinterpret_cast<float*>(reinterpret_cast<char*>(base) + byte_off) = v;
}

// Byte offset (from dy) of the gradient row of token t = seq * L + l, ~0 for no write (see
// MPArgs::seg_off); requires (rows of dy) * lddy * 4 < 2^32
__device__ __forceinline__ uint32_t dy_row_off(const MPArgs& g, int64_t seq, int l, uint64_t bits) {
  if (l >= g.L) return ~0u;
  const int64_t t = seq * g.L + l;
  if (!g.seg_off) return (uint32_t)(t * g.lddy * 4);
  if (!((bits >> l) & 1ull)) return ~0u;   // masked: exact zero, outside the CSR
  const int64_t u = g.yrows[t];
  const int64_t row = g.seg_off[u + 1] - g.seg_off[u] == 1 ? g.dyu_row0 + u : t;
  return (uint32_t)(row * g.lddy * 4);
}

__device__ __forceinline__ const float* yrow(const MPArgs& g, int l) {
  return reinterpret_cast<const float*>(reinterpret_cast<const char*>(g.y) + yrow_off(g, l));
}

__device__ __forceinline__ uint32_t row_byte_off(const MPArgs& g, int64_t tok) {
  return (uint32_t)((g.yrows ? g.yrows[tok] : tok) * g.ldy * 4);
}

__device__ __forceinline__ void stage_rows(const MPArgs& g, int64_t seq) {
  extern __shared__ uint32_t nr_mp_rows[];
  const int tid = threadIdx.x;
  if (tid < 32) nr_mp_rows[tid] = row_byte_off(g, seq * g.L + (tid < g.L ? tid : 0));
  __syncthreads();
}

__device__ __forceinline__ float drop_scale(const MPArgs& g, int64_t elem) {
  if (g.p_drop <= 0.f) return 1.f;
  return nr_dropout_keep(g.dkey, (uint32_t)elem, g.dthresh) ? 1.f / (1.f - g.p_drop) : 0.f;
}

__device__ __forceinline__ uint64_t token_bits(const MPArgs& g, int64_t seq) {
  const int lane = threadIdx.x & 63;
  const bool m = lane < g.L && nr_mask_at(g.mask, g.mask_dt, seq * g.L + lane);
  return __ballot(m);
}

// Loads this lane's half of key row c = lane & 31 for one head (see below for the order).
template <int DK, int NP>
__device__ __forceinline__ void load_krow(const MPArgs& g, int64_t seq, int head, float (&a)[DK / 2]) {
  const int lane = threadIdx.x & 63, c = lane & 31, h = lane >> 5;
  constexpr int HK = DK / 2;
  if constexpr (NP > 0) {
    // bf16 steps: a[8t + u] = K[c][16t + 8h + u] (step t's eight k-slots of this lane half)
    const bool ok = c < g.L;
    const float* kr = yrow(g, ok ? c : 0) + head * DK + 8 * h;
#pragma unroll
    for (int t = 0; t < DK / 16; ++t) {
#pragma unroll
      for (int q4 = 0; q4 < 2; ++q4) {
        const float4 v = *reinterpret_cast<const float4*>(kr + 16 * t + 4 * q4);
        float* d = a + 8 * t + 4 * q4;
        d[0] = ok ? v.x : 0.f; d[1] = ok ? v.y : 0.f; d[2] = ok ? v.z : 0.f; d[3] = ok ? v.w : 0.f;
      }
    }
  } else {
    // lane (c, h) takes the 16-B chunks 2*s4 + h of row c: the two halves of the wave read the
    // two halves of the same 32-B span (the k order inside S = K Kᵀ is free).  Rows past L are
    // clamped and zeroed by a select, never a branch: a branch around a load makes hipcc wait
    // for it at the join, serialising the whole load stream.
    const bool ok = c < g.L;
    const float* kr = yrow(g, ok ? c : 0) + head * DK + 4 * h;
#pragma unroll
    for (int s = 0; s < HK; s += 4) {
      const float4 v = *reinterpret_cast<const float4*>(kr + 2 * s);
      a[s] = ok ? v.x : 0.f; a[s + 1] = ok ? v.y : 0.f; a[s + 2] = ok ? v.z : 0.f; a[s + 3] = ok ? v.w : 0.f;
    }
  }
}

// Block kb (features 32 kb .. 32 kb + 31) of the wave's key rows into the transpose tile tw[row][33]
// from the lanes' half-rows in load_krow's order (lane (c, h) holds row c; rows past L are zero there)
template <int DK, int NP>
__device__ __forceinline__ void stage_kblock(const float (&a)[DK / 2], int kb, float* tw) {
  const int lane = threadIdx.x & 63, c = lane & 31, h = lane >> 5;
  if constexpr (NP > 0) {   // a[8t + u] = K[c][16t + 8h + u]: steps t = 2kb, 2kb + 1
#pragma unroll
    for (int t = 2 * kb; t < 2 * kb + 2; ++t)
#pragma unroll
      for (int u = 0; u < 8; ++u) tw[c * 33 + 16 * t + 8 * h + u - 32 * kb] = a[8 * t + u];
  } else {                  // a[4m + q] = K[c][8m + 4h + q]: chunks m = 4kb .. 4kb + 3
#pragma unroll
    for (int m = 4 * kb; m < 4 * kb + 4; ++m)
#pragma unroll
      for (int q = 0; q < 4; ++q) tw[c * 33 + 8 * m + 4 * h + q - 32 * kb] = a[4 * m + q];
  }
}

// S and P of one head for this lane's row c = lane & 31 from its key half-row a[];
// returns P in p[16] (C layout).
template <int DK, int NP>
__device__ __forceinline__ void head_probs_from(const MPArgs& g, uint64_t bits, const float (&a)[DK / 2],
                                                float (&p)[16]) {
  const int lane = threadIdx.x & 63, c = lane & 31, h = lane >> 5;
  constexpr int HK = DK / 2;
  f32x16 S;
#pragma unroll
  for (int r = 0; r < 16; ++r) S[r] = 0.f;
  if constexpr (NP == 0) {
#pragma unroll
    for (int s = 0; s < HK; ++s) S = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], a[s], S, 0, 0, 0);
  } else {   // K is both operands: the lane's own key chunk, split once
#pragma unroll
    for (int t = 0; t < DK / 16; ++t) {
      const Planes<NP> pk = planes8<NP>(a + 8 * t);
      mfma_x<NP>(S, pk, pk);
    }
  }
  const bool mj = (bits >> c) & 1ull;
  float mx = -INFINITY;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const bool keep = mj && ((bits >> crow(r, h)) & 1ull);
    p[r] = keep ? S[r] * g.scale_attn : -INFINITY;
    mx = fmaxf(mx, p[r]);
  }
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  float sum = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const float e = p[r] == -INFINITY ? 0.f : __expf(p[r] - mx);
    p[r] = e;
    sum += e;
  }
  sum += __shfl_xor(sum, 32, 64);
  const float inv = sum > 0.f ? 1.f / sum : 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) p[r] *= inv;
}

// V operand of O = P V: lane (c, h) needs V[crow(s, h)][vb*32 + c] (rows past L -> 0)
template <int DK, int DV>
__device__ __forceinline__ void load_vop(const MPArgs& g, int64_t seq, int head, float (&bv)[DV / 2]) {
  const int lane = threadIdx.x & 63, c = lane & 31, h = lane >> 5;
  const int nq = g.heads * DK;
#pragma unroll
  for (int vb = 0; vb < DV / 32; ++vb)
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int k = crow(s, h);
      const float v = ld_off(g.y, yrow_off(g, k < g.L ? k : 0) + 4u * (uint32_t)(nq + head * DV + vb * 32 + c));
      bv[vb * 16 + s] = k < g.L ? v : 0.f;
    }
}

// O_h = P V_h into the LDS image os[32][so] at columns head*DV ..
template <int DK, int DV, int NP>
__device__ __forceinline__ void head_out(const float (&bv)[DV / 2], int head, const float (&p)[16], float* os,
                                         int so) {
  const int lane = threadIdx.x & 63, c = lane & 31, h = lane >> 5;
#pragma unroll
  for (int vb = 0; vb < DV / 32; ++vb) {
    f32x16 O;
#pragma unroll
    for (int r = 0; r < 16; ++r) O[r] = 0.f;
    mfma16<NP>(O, p, bv + vb * 16);
#pragma unroll
    for (int r = 0; r < 16; ++r) os[crow(r, h) * so + head * DV + vb * 32 + c] = O[r];
  }
}

template <int DK, int DV, int NP>
__device__ void attention_to_lds(const MPArgs& g, int64_t seq, uint64_t bits, float* os, int so) {
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if (nw < g.heads) {
    // several heads per wave (the four-wave forward): the next head's key / value loads are issued
    // before this head's products, so each load latency hides behind the previous head's work.
    // Heads w, w + nw, w + 2 nw; a prefetch past the last head re-reads the last one (clamped, no
    // branch around a load: hipcc would wait for it at the join).
    float a0[DK / 2], b0[DV / 2], a1[DK / 2], b1[DV / 2];
    const int hl = g.heads - 1;
    const int h0 = w, h1 = w + nw, h2 = w + 2 * nw;
    load_krow<DK, NP>(g, seq, h0 < hl ? h0 : hl, a0);
    load_vop<DK, DV>(g, seq, h0 < hl ? h0 : hl, b0);
    load_krow<DK, NP>(g, seq, h1 < hl ? h1 : hl, a1);
    load_vop<DK, DV>(g, seq, h1 < hl ? h1 : hl, b1);
    float p[16];
    if (h0 <= hl) {
      head_probs_from<DK, NP>(g, bits, a0, p);
      head_out<DK, DV, NP>(b0, h0, p, os, so);
    }
    load_krow<DK, NP>(g, seq, h2 < hl ? h2 : hl, a0);
    load_vop<DK, DV>(g, seq, h2 < hl ? h2 : hl, b0);
    if (h1 <= hl) {
      head_probs_from<DK, NP>(g, bits, a1, p);
      head_out<DK, DV, NP>(b1, h1, p, os, so);
    }
    if (h2 <= hl) {
      head_probs_from<DK, NP>(g, bits, a0, p);
      head_out<DK, DV, NP>(b0, h2, p, os, so);
    }
    for (int head = w + 3 * nw; head < g.heads; head += nw) {   // more than three heads per wave
      load_krow<DK, NP>(g, seq, head, a0);
      load_vop<DK, DV>(g, seq, head, b0);
      head_probs_from<DK, NP>(g, bits, a0, p);
      head_out<DK, DV, NP>(b0, head, p, os, so);
    }
    return;
  }
  for (int head = w; head < g.heads; head += nw) {
    // issue the key and value loads together: one memory latency per head, not two
    float a[DK / 2], bv[DV / 2];
    load_krow<DK, NP>(g, seq, head, a);
    load_vop<DK, DV>(g, seq, head, bv);
    float p[16];
    head_probs_from<DK, NP>(g, bits, a, p);
    head_out<DK, DV, NP>(bv, head, p, os, so);
  }}

template <int DK, int DV, int NH64, int NP>
__global__ __launch_bounds__(768) void mha_pool_fwd_kernel(MPArgs g) {
  if (g.rng) g.dkey = nr_dropout_key(g.rng[0], g.rng[1] + g.offset);   // graph-replay RNG
  extern __shared__ __attribute__((aligned(16))) float sm[];
  constexpr int H = NH64 * 64;
  constexpr int SO = H + 1;
  float* os = sm + 32;                  // [32][SO]  O, then Z (sm[0..32): staged rows, yrow)
  float* sc = os + 32 * SO;             // [32] scores -> probs
  const int64_t seq = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, nw = blockDim.x >> 6, nt = blockDim.x;
  const uint64_t bits = token_bits(g, seq);
  stage_rows(g, seq);
  attention_to_lds<DK, DV, NP>(g, seq, bits, os, SO);
  // the LayerNorm / pooling vectors are loaded only now: held through the attention phase they
  // would raise its register peak (and so lower the titles in flight per CU)
  float gam[NH64], bet[NH64], qv[NH64];
#pragma unroll
  for (int k = 0; k < NH64; ++k) {
    gam[k] = g.gamma[lane + 64 * k];
    bet[k] = g.beta[lane + 64 * k];
    qv[k] = g.q[lane + 64 * k];
  }
  __syncthreads();
  // LayerNorm + dropout in place, scores; one wave per row
  for (int l = w; l < g.L; l += nw) {
    const int64_t row = seq * g.L + l;
    float x[NH64];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NH64; ++k) { x[k] = os[l * SO + lane + 64 * k]; s += x[k]; }
    if (g.o) {   // saved attention output for the split backward
#pragma unroll
      for (int k = 0; k < NH64; ++k) g.o[row * g.ldo + lane + 64 * k] = x[k];
    }
    const float mean = nr_wave_sum(s) * (1.f / H);
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < NH64; ++k) { const float d = x[k] - mean; v = fmaf(d, d, v); }
    const float rstd = rsqrtf(nr_wave_sum(v) * (1.f / H) + g.eps);
    float dot = 0.f;
#pragma unroll
    for (int k = 0; k < NH64; ++k) {
      const int d = lane + 64 * k;
      const float z = ((x[k] - mean) * rstd * gam[k] + bet[k]) * drop_scale(g, row * H + d);
      os[l * SO + d] = z;
      if (g.zout) g.zout[row * g.ldz + d] = z;
      dot = fmaf(qv[k], z, dot);
    }
    dot = nr_wave_sum(dot);
    if (lane == 0) {
      g.stats[2 * row] = mean;
      g.stats[2 * row + 1] = rstd;
      sc[l] = dot * g.scale_pool;
    }
  }
  __syncthreads();
  if (w == 0) {
    const bool keep = lane < 32 && ((bits >> lane) & 1ull);
    const float v = keep ? sc[lane & 31] : -INFINITY;
    const float mx = nr_wave_max(v);
    const float e = keep ? __expf(v - mx) : 0.f;
    const float sum = nr_wave_sum(e);
    const float pr = sum > 0.f ? e / sum : 0.f;
    if (lane < g.L) {
      sc[lane] = pr;
      g.probs[seq * g.L + lane] = pr;
    }
  }
  __syncthreads();
  for (int d = tid; d < H; d += nt) {
    float acc = 0.f;
    for (int l = 0; l < g.L; ++l) acc = fmaf(sc[l], os[l * SO + d], acc);
    g.news[seq * g.ldn + d] = acc;
  }
}

// Pooling + dropout + LayerNorm backward of one title.  On entry os[l][*] holds the attention
// output O rows (rows >= L zero), ps / st the saved pooling probabilities and LN (mean, rstd).
// On exit os holds dO (rows < L; rows >= L untouched); dq, dgamma, dbeta accumulate
// atomically; dob (optional) receives the dO rows in global memory too.  Two row passes, one
// wave per row: (1) dp_l = dnews · Z_l, keeping the row's dropout keep-bits in LDS (one hash
// per element for the whole backward); (2) after the pooling-softmax backward, dZ -> dropout ->
// LayerNorm backward with per-lane partials of dq, dgamma, dbeta, reduced across the waves
// through `red` ([nw][3][H]; may alias scratch that is free until the trailing barrier).
template <int NH64>
__device__ __forceinline__ void pool_ln_bwd(const MPArgs& g, int64_t seq, float* os, const float* ps, float* ds,
                                            const float* st, float* red, uint64_t* kbits, float* dob,
                                            int64_t lddob) {
  constexpr int H = NH64 * 64;
  constexpr int SO = H + 1;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, nw = blockDim.x >> 6, nt = blockDim.x;
  const bool drop = g.p_drop > 0.f;
  const float dsc = drop ? 1.f / (1.f - g.p_drop) : 1.f;
  float gam[NH64], bet[NH64], qv[NH64], dnv[NH64];
#pragma unroll
  for (int k = 0; k < NH64; ++k) {
    gam[k] = g.gamma[lane + 64 * k];
    bet[k] = g.beta[lane + 64 * k];
    qv[k] = g.q[lane + 64 * k];
    dnv[k] = g.news[seq * g.ldn + lane + 64 * k];
  }
  // (1) dp_l = dnews · Z_l; keep-bits of row l -> kbits[l][k]
  for (int l = w; l < g.L; l += nw) {
    const int64_t row = seq * g.L + l;
    const float mean = st[2 * l], rstd = st[2 * l + 1];
    float dot = 0.f;
#pragma unroll
    for (int k = 0; k < NH64; ++k) {
      const int d = lane + 64 * k;
      const bool keep = !drop || nr_dropout_keep(g.dkey, (uint32_t)(row * H + d), g.dthresh);
      const uint64_t b = __ballot(keep);
      if (lane == 0) kbits[l * NH64 + k] = b;
      const float z = keep ? ((os[l * SO + d] - mean) * rstd * gam[k] + bet[k]) * dsc : 0.f;
      dot = fmaf(dnv[k], z, dot);
    }
    dot = nr_wave_sum(dot);
    if (lane == 0) ds[l] = dot;
  }
  __syncthreads();
  if (w == 0) {   // pooling softmax backward: ds_l = p_l (dp_l - Σ p dp) / sqrt(H)
    const float pl = lane < 32 ? ps[lane & 31] : 0.f;
    const float dp = lane < g.L ? ds[lane & 31] : 0.f;
    const float r = nr_wave_sum(pl * dp);
    if (lane < g.L) ds[lane] = pl * (dp - r) * g.scale_pool;
  }
  __syncthreads();
  // (2) dq += ds_l Z_l;  dZ = p_l dnews + ds_l q (+ dz) -> dropout -> LayerNorm backward
  float dgam[NH64], dbet[NH64], dqp[NH64];
#pragma unroll
  for (int k = 0; k < NH64; ++k) { dgam[k] = 0.f; dbet[k] = 0.f; dqp[k] = 0.f; }
  for (int l = w; l < g.L; l += nw) {
    const int64_t row = seq * g.L + l;
    const float mean = st[2 * l], rstd = st[2 * l + 1], pl = ps[l], dsl = ds[l];
    float xh[NH64], dyv[NH64];
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int k = 0; k < NH64; ++k) {
      const int d = lane + 64 * k;
      const float s = ((kbits[l * NH64 + k] >> lane) & 1ull) ? dsc : 0.f;
      xh[k] = (os[l * SO + d] - mean) * rstd;
      dqp[k] = fmaf(dsl, (xh[k] * gam[k] + bet[k]) * s, dqp[k]);
      float dz = fmaf(pl, dnv[k], dsl * qv[k]);
      if (g.dz) dz += g.dz[row * g.lddz + d];
      dyv[k] = dz * s;
      const float gg = dyv[k] * gam[k];
      sg += gg;
      sgx = fmaf(gg, xh[k], sgx);
      dgam[k] = fmaf(dyv[k], xh[k], dgam[k]);
      dbet[k] += dyv[k];
    }
    sg = nr_wave_sum(sg) * (1.f / H);
    sgx = nr_wave_sum(sgx) * (1.f / H);
#pragma unroll
    for (int k = 0; k < NH64; ++k) {
      const int d = lane + 64 * k;
      const float v = rstd * (dyv[k] * gam[k] - sg - xh[k] * sgx);
      os[l * SO + d] = v;
      if (dob) dob[row * lddob + d] = v;
    }
  }
#pragma unroll
  for (int k = 0; k < NH64; ++k) {
    red[(w * 3) * H + lane + 64 * k] = dgam[k];
    red[(w * 3 + 1) * H + lane + 64 * k] = dbet[k];
    red[(w * 3 + 2) * H + lane + 64 * k] = dqp[k];
  }
  __syncthreads();
  for (int d = tid; d < H; d += nt) {
    float a = 0.f, b = 0.f, q = 0.f;
    for (int ww = 0; ww < nw; ++ww) {
      a += red[(ww * 3) * H + d];
      b += red[(ww * 3 + 1) * H + d];
      q += red[(ww * 3 + 2) * H + d];
    }
    atomicAdd(g.ws ? grad_slot(g, d) : &g.dgamma[d], a);
    atomicAdd(g.ws ? grad_slot(g, H + d) : &g.dbeta[d], b);
    atomicAdd(g.ws ? grad_slot(g, 2 * H + d) : &g.dq[d], q);
  }
  __syncthreads();   // red may alias later scratch
}

// dO of one head for the attention backward: from the workgroup's LDS image (fused kernel:
// rows >= L are zero there) or from the global dO rows (split form: clamp + zero by select).
template <int DV>
struct DoSource {
  const float* base;   // row 0, column head*DV
  int64_t ld;
  int L;
  bool global;
  __device__ __forceinline__ float at(int l, int col) const {
    if (!global) return base[l * ld + col];
    const float v = ld_off(base, 4u * (uint32_t)((l < L ? l : 0) * (int)ld + col));
    return l < L ? v : 0.f;
  }
};

// Attention backward of one (title, head) by one wave (the title's projection rows staged by
// stage_rows*): recompute P from the key rows, dV = Pᵀ dO, dPᵀ = V dOᵀ, dS (XSoftmax
// backward), W = dS + dSᵀ (tied Q = K), dK = W K; dV / dK rows to dy, their column sums added
// to cs[] (dbias: cs[vb] for the value columns, cs[DV/32 + kb] for the key columns).
template <int DK, int DV, int NP>
__device__ __forceinline__ void head_bwd(const MPArgs& g, int64_t seq, int head, uint64_t bits, float* tw,
                                         const DoSource<DV>& dO, float (&cs)[DV / 32 + DK / 32],
                                         const uint32_t* dsto) {
  const int lane = threadIdx.x & 63, c = lane & 31, h = lane >> 5;
  const int nq = g.heads * DK;

  float p[16];
  float ka[DK / 2];   // this lane's key half-row, kept for dK = W K (staged through tw, not re-loaded)
  load_krow<DK, NP>(g, seq, head, ka);
  head_probs_from<DK, NP>(g, bits, ka, p);
  // phase fences: keep each phase's loads inside it (hoisting them all to the top costs more
  // registers than the latency they would hide; the split kernel runs 4 waves per SIMD)
  __builtin_amdgcn_sched_barrier(0);
  // dVp = Pᵀ dO first (P is live anyway): Pᵀ through the transpose tile
  {
#pragma unroll
    for (int r = 0; r < 16; ++r) tw[c * 33 + crow(r, h)] = p[r];
    wave_lds_fence();
    float pt[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) pt[s] = tw[crow(s, h) * 33 + c];
    wave_lds_fence();
#pragma unroll
    for (int vb = 0; vb < DV / 32; ++vb) {
      float bo[16];
#pragma unroll
      for (int s = 0; s < 16; ++s) bo[s] = dO.at(crow(s, h), vb * 32 + c);
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
      mfma16<NP>(acc, pt, bo);
      float sum = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = crow(r, h);
        if (i < g.L && dsto[i] != ~0u) st_off(g.dy, dsto[i] + 4u * (uint32_t)(nq + head * DV + vb * 32 + c), acc[r]);
        sum += acc[r];
      }
      cs[vb] += sum;
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // dPᵀ = V dOᵀ  (lane (c, h): V[c][k], dO[c][k] over the interleaved k order)
  float dsv[16];
  {
    f32x16 dpt;
#pragma unroll
    for (int r = 0; r < 16; ++r) dpt[r] = 0.f;
    constexpr int HV = DV / 2;
    const bool rv = c < g.L;
    if constexpr (NP == 0) {
      const float* vrr = yrow(g, rv ? c : 0) + nq + head * DV + 4 * h;   // clamp, zero by select
#pragma unroll
      for (int s = 0; s < HV; s += 4) {
        float4 v4 = *reinterpret_cast<const float4*>(vrr + 2 * s);
        if (!rv) v4 = make_float4(0.f, 0.f, 0.f, 0.f);
        const int col = 4 * h + 2 * s;
        dpt = __builtin_amdgcn_mfma_f32_32x32x2f32(v4.x, dO.at(c, col), dpt, 0, 0, 0);
        dpt = __builtin_amdgcn_mfma_f32_32x32x2f32(v4.y, dO.at(c, col + 1), dpt, 0, 0, 0);
        dpt = __builtin_amdgcn_mfma_f32_32x32x2f32(v4.z, dO.at(c, col + 2), dpt, 0, 0, 0);
        dpt = __builtin_amdgcn_mfma_f32_32x32x2f32(v4.w, dO.at(c, col + 3), dpt, 0, 0, 0);
      }
    } else {   // features 16t + 8h + u of V row c and dO row c
      const float* vrr = yrow(g, rv ? c : 0) + nq + head * DV + 8 * h;
#pragma unroll
      for (int t = 0; t < DV / 16; ++t) {
        float va[8], oa[8];
#pragma unroll
        for (int q4 = 0; q4 < 2; ++q4) {
          const float4 v4 = *reinterpret_cast<const float4*>(vrr + 16 * t + 4 * q4);
          va[4 * q4] = rv ? v4.x : 0.f; va[4 * q4 + 1] = rv ? v4.y : 0.f;
          va[4 * q4 + 2] = rv ? v4.z : 0.f; va[4 * q4 + 3] = rv ? v4.w : 0.f;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) oa[u] = dO.at(c, 16 * t + 8 * h + u);
        mfma_x<NP>(dpt, planes8<NP>(va), planes8<NP>(oa));
      }
    }
    float rs = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) rs = fmaf(p[r], dpt[r], rs);
    rs += __shfl_xor(rs, 32, 64);
#pragma unroll
    for (int r = 0; r < 16; ++r) dsv[r] = p[r] * (dpt[r] - rs) * g.scale_attn;
  }
  __builtin_amdgcn_sched_barrier(0);
  // W = dS + dSᵀ via the per-wave transpose tile
#pragma unroll
  for (int r = 0; r < 16; ++r) tw[c * 33 + crow(r, h)] = dsv[r];
  wave_lds_fence();
#pragma unroll
  for (int r = 0; r < 16; ++r) dsv[r] += tw[crow(r, h) * 33 + c];
  wave_lds_fence();
  // dKp = W Kp  -> dY[:, head*DK ..]; K's 32-feature block kb from the lanes' key rows through tw
#pragma unroll
  for (int kb = 0; kb < DK / 32; ++kb) {
    stage_kblock<DK, NP>(ka, kb, tw);
    wave_lds_fence();
    float bk[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) bk[s] = tw[crow(s, h) * 33 + c];
    wave_lds_fence();
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    mfma16<NP>(acc, dsv, bk);
    float sum = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int j = crow(r, h);
      if (j < g.L && dsto[j] != ~0u) st_off(g.dy, dsto[j] + 4u * (uint32_t)(head * DK + kb * 32 + c), acc[r]);
      sum += acc[r];
    }
    cs[DV / 32 + kb] += sum;
    __builtin_amdgcn_sched_barrier(0);
  }
}

// dbias column sums of one head: lanes of the two halves hold partial sums of the same column
template <int DK, int DV>
__device__ __forceinline__ void flush_dbias(const MPArgs& g, int head, float (&cs)[DV / 32 + DK / 32]) {
  const int lane = threadIdx.x & 63, c = lane & 31, h = lane >> 5;
  const int nq = g.heads * DK;
#pragma unroll
  for (int i = 0; i < DV / 32 + DK / 32; ++i) {
    const float v = cs[i] + __shfl_xor(cs[i], 32, 64);
    const int col = i < DV / 32 ? nq + head * DV + i * 32 + c : head * DK + (i - DV / 32) * 32 + c;
    if (h == 0) atomicAdd(g.ws ? grad_slot(g, 3 * (int64_t)g.heads * DV + col) : &g.dbias[col], v);
    cs[i] = 0.f;
  }
}

// Fused backward: the attention output O into LDS -- recomputed from the projections, or (SAVED)
// the rows the training forward saved -- then the pooling/LN backward in place and the attention
// backward of every head with dO from LDS.  SAVED keeps dO on chip (the split form writes it to HBM
// and reads it back, 2 x 81 MB per NRMS step).
template <int DK, int DV, int NH64, int NP, bool SAVED>
__global__ __launch_bounds__(384) void mha_pool_bwd_kernel(MPArgs g) {
  if (g.rng) g.dkey = nr_dropout_key(g.rng[0], g.rng[1] + g.offset);   // graph-replay RNG
  extern __shared__ __attribute__((aligned(16))) float sm[];
  constexpr int H = NH64 * 64;
  constexpr int SO = H + 1;
  const int nw = blockDim.x >> 6;
  float* os = sm + 32;                  // [32][SO]  O, then dO (sm[0..32): staged rows, yrow)
  float* ps = os + 32 * SO;             // [32] pooling probs
  float* ds = ps + 32;                  // [32] dp -> ds
  float* st = ds + 32;                  // [32][2] mean, rstd
  uint64_t* kb = reinterpret_cast<uint64_t*>(st + 64);   // [32][NH64] dropout keep-bits
  float* ts = st + 64 + 2 * 32 * NH64;  // [nw][32][33] per-wave transpose tiles
  float* red = ts;                      // [nw][3][H] dgamma / dbeta / dq partials (before ts is used)
  const int64_t seq = blockIdx.x;
  const int tid = threadIdx.x, w = tid >> 6;
  const uint64_t bits = token_bits(g, seq);
  stage_rows(g, seq);
  if constexpr (SAVED) {
    constexpr int H4 = NH64 * 16;   // float4 per O row
    for (int i = tid; i < 32 * H4; i += blockDim.x) {
      const int l = i / H4, c4 = i - l * H4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (l < g.L) v = *reinterpret_cast<const float4*>(g.o + (seq * g.L + l) * g.ldo + 4 * c4);
      float* d = os + l * SO + 4 * c4;
      d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
    }
  } else {
    attention_to_lds<DK, DV, NP>(g, seq, bits, os, SO);
  }
  if (tid < 32) {
    ps[tid] = tid < g.L ? g.probs[seq * g.L + tid] : 0.f;
    st[2 * tid] = tid < g.L ? g.stats[2 * (seq * g.L + tid)] : 0.f;
    st[2 * tid + 1] = tid < g.L ? g.stats[2 * (seq * g.L + tid) + 1] : 0.f;
  }
  __syncthreads();
  __shared__ uint32_t s_dsto[32];
  if (tid < 32) s_dsto[tid] = dy_row_off(g, seq, tid, bits);
  pool_ln_bwd<NH64>(g, seq, os, ps, ds, st, red, kb, nullptr, 0);   // (its barriers publish s_dsto)
  float* tw = ts + w * 32 * 33;
  for (int head = w; head < g.heads; head += nw) {
    DoSource<DV> dO{os + head * DV, SO, g.L, false};
    float cs[DV / 32 + DK / 32];
#pragma unroll
    for (int i = 0; i < DV / 32 + DK / 32; ++i) cs[i] = 0.f;
    head_bwd<DK, DV, NP>(g, seq, head, bits, tw, dO, cs, s_dsto);
    flush_dbias<DK, DV>(g, head, cs);
  }
}

// One element of the LayerNorm / dropout / pooling backward, dO = rstd (dyv γ - sg - x̂ sgx) with
// x̂ = (O - mean) rstd and dyv = (p_l dnews + ds_l q (+ dz)) · keep / (1 - p): the split backward's LN
// pass (mha_ln_bwd_kernel) forms the row terms, the head pass (mha_head_bwd_kernel) the elements of its
// head's columns, both through this function (the same operations in the same order).
__device__ __forceinline__ float ln_row_dO(float xh, float rstd, float sg, float sgx, float pl, float dsl, float dn,
                                           float qd, float gm, float dzv, float sk) {
  const float dyv = (fmaf(pl, dn, dsl * qd) + dzv) * sk;
  return rstd * fmaf(-xh, sgx, fmaf(dyv, gm, -sg));
}

// Split backward, kernel 1 (forward saved O): pooling/LN backward per title from the saved O
// rows; the per-row terms of dO to global ([T][8]: mean, rstd, sg, sgx, ds_l, p_l).  Register-resident:
// wave w owns rows w, w + 4, ... of the title and keeps
// them (and their dropout keep-bits) in registers through both passes; only the 32 pooling scores
// and the cross-wave dgamma / dbeta / dq partials go through LDS (~19 KB instead of ~68 KB staging
// the whole O tile, so several titles share a CU and their loads overlap).
template <int NH64>
__global__ __launch_bounds__(256) void mha_ln_bwd_kernel(MPArgs g) {
  if (g.rng) g.dkey = nr_dropout_key(g.rng[0], g.rng[1] + g.offset);   // graph-replay RNG
  constexpr int H = NH64 * 64;
  constexpr int RW = 8;                 // rows per wave (L <= 32, 4 waves)
  __shared__ float sdp[32], sps[32];
  __shared__ float red[4][3][H];
  const int64_t seq = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int L = g.L;
  const bool drop = g.p_drop > 0.f;
  const float dsc = drop ? 1.f / (1.f - g.p_drop) : 1.f;
  float x[RW][NH64];
  // every O load of the wave in flight at once (rows past L clamped, their values unused)
#pragma unroll
  for (int i = 0; i < RW; ++i) {
    const int l = w + 4 * i;
    const float* orow = g.o + (seq * L + (l < L ? l : 0)) * g.ldo;
#pragma unroll
    for (int k = 0; k < NH64; ++k) x[i][k] = orow[lane + 64 * k];
  }
  float gam[NH64], bet[NH64], qv[NH64], dnv[NH64];
#pragma unroll
  for (int k = 0; k < NH64; ++k) {
    gam[k] = g.gamma[lane + 64 * k];
    bet[k] = g.beta[lane + 64 * k];
    qv[k] = g.q[lane + 64 * k];
    dnv[k] = g.news[seq * g.ldn + lane + 64 * k];
  }
  if (tid < 32) sps[tid] = tid < L ? g.probs[seq * L + tid] : 0.f;
  if (g.dsto && tid < L) g.dsto[seq * L + tid] = dy_row_off(g, seq, tid, token_bits(g, seq));
  // (1) normalise in place (x -> x_hat), dp_l = dnews · Z_l, keep-bits kept per row
  static_assert(NH64 <= 32, "keep-bits of a row fit one word");
  uint32_t kbit[RW];
#pragma unroll
  for (int i = 0; i < RW; ++i) {
    const int l = w + 4 * i;
    kbit[i] = 0;
    if (l >= L) continue;
    const int64_t row = seq * L + l;
    const float mean = g.stats[2 * row], rstd = g.stats[2 * row + 1];
    float dot = 0.f;
    uint32_t kb = 0;
#pragma unroll
    for (int k = 0; k < NH64; ++k) {
      const int d = lane + 64 * k;
      const bool keep = !drop || nr_dropout_keep(g.dkey, (uint32_t)(row * H + d), g.dthresh);
      kb |= (keep ? 1u : 0u) << k;
      x[i][k] = (x[i][k] - mean) * rstd;
      const float z = keep ? (x[i][k] * gam[k] + bet[k]) * dsc : 0.f;
      dot = fmaf(dnv[k], z, dot);
    }
    kbit[i] = kb;
    dot = nr_wave_sum(dot);
    if (lane == 0) sdp[l] = dot;
  }
  __syncthreads();
  if (w == 0) {   // pooling softmax backward: ds_l = p_l (dp_l - Σ p dp) / sqrt(H)
    const float pl = lane < 32 ? sps[lane & 31] : 0.f;
    const float dp = lane < L ? sdp[lane & 31] : 0.f;
    const float r = nr_wave_sum(pl * dp);
    if (lane < L) sdp[lane] = pl * (dp - r) * g.scale_pool;
  }
  __syncthreads();
  // (2) dq += ds_l Z_l;  dZ = p_l dnews + ds_l q (+ dz) -> dropout -> LayerNorm backward -> dO
  float dgam[NH64], dbet[NH64], dqp[NH64];
#pragma unroll
  for (int k = 0; k < NH64; ++k) { dgam[k] = 0.f; dbet[k] = 0.f; dqp[k] = 0.f; }
#pragma unroll
  for (int i = 0; i < RW; ++i) {
    const int l = w + 4 * i;
    if (l >= L) continue;
    const int64_t row = seq * L + l;
    const float rstd = g.stats[2 * row + 1], pl = sps[l], dsl = sdp[l];
    float dyv[NH64];
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int k = 0; k < NH64; ++k) {
      const int d = lane + 64 * k;
      const float sk = ((kbit[i] >> k) & 1u) ? dsc : 0.f;
      dqp[k] = fmaf(dsl, (x[i][k] * gam[k] + bet[k]) * sk, dqp[k]);
      // dyv exactly as ln_row_dO forms it in the head pass
      dyv[k] = (fmaf(pl, dnv[k], dsl * qv[k]) + (g.dz ? g.dz[row * g.lddz + d] : 0.f)) * sk;
      const float gg = dyv[k] * gam[k];
      sg += gg;
      sgx = fmaf(gg, x[i][k], sgx);
      dgam[k] = fmaf(dyv[k], x[i][k], dgam[k]);
      dbet[k] += dyv[k];
    }
    sg = nr_wave_sum(sg) * (1.f / H);
    sgx = nr_wave_sum(sgx) * (1.f / H);
    // the row's terms of dO = rstd (dyv γ - sg - x̂ sgx): the head pass rebuilds its slice of dO from
    // the saved O with them (ln_row_dO), so the [T, H] dO never goes through HBM
    if (lane == 0) {
      float4* rc = reinterpret_cast<float4*>(g.dob + row * g.lddob);
      rc[0] = make_float4(g.stats[2 * row], rstd, sg, sgx);
      rc[1] = make_float4(dsl, pl, 0.f, 0.f);
    }
  }
#pragma unroll
  for (int k = 0; k < NH64; ++k) {
    red[w][0][lane + 64 * k] = dgam[k];
    red[w][1][lane + 64 * k] = dbet[k];
    red[w][2][lane + 64 * k] = dqp[k];
  }
  __syncthreads();
  float* ogam = g.ws ? grad_slot(g, 0) : g.dgamma;
  float* obet = g.ws ? grad_slot(g, H) : g.dbeta;
  float* oq = g.ws ? grad_slot(g, 2 * H) : g.dq;
  for (int d = tid; d < H; d += 256) {
    atomicAdd(&ogam[d], (red[0][0][d] + red[1][0][d]) + (red[2][0][d] + red[3][0][d]));
    atomicAdd(&obet[d], (red[0][1][d] + red[1][1][d]) + (red[2][1][d] + red[3][1][d]));
    atomicAdd(&oq[d], (red[0][2][d] + red[1][2][d]) + (red[2][2][d] + red[3][2][d]));
  }
}

// Split backward, kernel 2: attention backward, one wave per head, HB_TITLES titles per
// workgroup in sequence (the dbias column sums accumulate in registers across them: one
// atomic per column per workgroup instead of per title).  Each wave stages its title's
// projection-row indices in a private slice of LDS.
constexpr int HB_TITLES = 1;

template <int DK, int DV, int NP>
__global__ __launch_bounds__(256, 4) void mha_head_bwd_kernel(MPArgs g) {
  if (g.rng) g.dkey = nr_dropout_key(g.rng[0], g.rng[1] + g.offset);   // graph-replay RNG (dO's dropout)
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int head = blockIdx.y * nw + w;
  if (head >= g.heads) return;   // no block-wide barrier below
  uint32_t* rows = reinterpret_cast<uint32_t*>(sm) + 32 * w;   // this wave's staged row offsets (yrow)
  uint32_t* dsts = reinterpret_cast<uint32_t*>(sm) + 32 * nw + 32 * w;   // ... and dy row offsets
  float* tw = sm + 64 * nw + w * 32 * 33;                     // this wave's transpose tile
  float* dot = sm + 64 * nw + nw * 32 * 33 + w * 32 * (DV + 1);   // this wave's dO slice [32][DV+1]
  float cs[DV / 32 + DK / 32];
#pragma unroll
  for (int i = 0; i < DV / 32 + DK / 32; ++i) cs[i] = 0.f;
  const int64_t s0 = (int64_t)blockIdx.x * HB_TITLES;
#pragma unroll 1
  for (int64_t seq = s0; seq < s0 + HB_TITLES && seq < g.nseq; ++seq) {
    // every global load of the prologue in flight together: row ids, mask, the head's dO slice
    const uint32_t roff = lane < 32 ? row_byte_off(g, seq * g.L + (lane < g.L ? lane : 0)) : 0u;
    const uint64_t bits = token_bits(g, seq);
    uint32_t doff = ~0u;
    if (lane < g.L) doff = g.dsto ? g.dsto[seq * g.L + lane] : (uint32_t)((seq * g.L + lane) * g.lddy * 4);
    constexpr int F4 = DV / 4;                 // float4 per dO row
    constexpr int PER = 32 * F4 / 64;          // per lane
    static_assert(64 % F4 == 0, "a lane keeps its four columns in every row it loads");
    // this head's slice of dO, rebuilt from the saved attention output O and the LN pass's row terms
    // (ln_row_dO: the dO rows never go through HBM); lane: rows e / F4 of e = lane + 64 i, columns
    // 4 (lane % F4) .. + 3 of the head
    float4 v[PER], ra[PER], rb[PER];
    const int col0 = head * DV + 4 * (lane % F4);
    {
      const float* src = g.o + (seq * g.L) * g.ldo + head * DV;
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int e = lane + 64 * i, r = e / F4, c4 = e % F4;
        const int rr = r < g.L ? r : 0;
        v[i] = *reinterpret_cast<const float4*>(
            reinterpret_cast<const char*>(src) + 4u * (uint32_t)(rr * (int)g.ldo + 4 * c4));
        const float4* rc = reinterpret_cast<const float4*>(g.dob + (seq * g.L + rr) * g.lddob);
        ra[i] = rc[0];   // mean, rstd, sg, sgx
        rb[i] = rc[1];   // ds_l, p_l
      }
    }
    float gm[4], qd[4], dn[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      gm[j] = g.gamma[col0 + j];
      qd[j] = g.q[col0 + j];
      dn[j] = g.news[seq * g.ldn + col0 + j];
    }
    {
      const bool drop = g.p_drop > 0.f;
      const float dsc = drop ? 1.f / (1.f - g.p_drop) : 1.f;
      const uint32_t Hc = (uint32_t)(g.heads * DV);
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int r = (lane + 64 * i) / F4;
        const int64_t row = seq * g.L + (r < g.L ? r : 0);
        float o[4] = {v[i].x, v[i].y, v[i].z, v[i].w}, d[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t col = (uint32_t)(col0 + j);
          const bool keep = !drop || nr_dropout_keep(g.dkey, (uint32_t)row * Hc + col, g.dthresh);
          const float dzv = g.dz ? g.dz[row * g.lddz + col] : 0.f;
          const float xh = (o[j] - ra[i].x) * ra[i].y;
          d[j] = ln_row_dO(xh, ra[i].y, ra[i].z, ra[i].w, rb[i].y, rb[i].x, dn[j], qd[j], gm[j], dzv,
                           keep ? dsc : 0.f);
        }
        v[i] = r < g.L ? make_float4(d[0], d[1], d[2], d[3]) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
    if (lane < 32) {
      rows[lane] = roff;
      dsts[lane] = doff;
    }
#pragma unroll
    for (int i = 0; i < PER; ++i) {   // dO slice into LDS, rows >= L zero
      const int e = lane + 64 * i, r = e / F4, c4 = e % F4;
      float* d = dot + r * (DV + 1) + 4 * c4;
      d[0] = v[i].x; d[1] = v[i].y; d[2] = v[i].z; d[3] = v[i].w;
    }
    wave_lds_fence();
    DoSource<DV> dO{dot, DV + 1, g.L, false};
    head_bwd<DK, DV, NP>(g, seq, head, bits, tw, dO, cs, dsts);
    wave_lds_fence();   // the next title's row indices / dO overwrite these
  }
  flush_dbias<DK, DV>(g, head, cs);
}

// out[i] += Σ_c ws[c][i] over the copies, each copy re-zeroed (the workspace is left zero for the
// next call); columns [0,H) dgamma, [H,2H) dbeta, [2H,3H) dq, [3H, 3H+NY) dbias
__global__ __launch_bounds__(64) void copies_reduce_kernel(MPArgs g, int H, int NY) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  if (i >= 3 * H + NY) return;
  float s = 0.f;
  for (int c0 = 0; c0 < g.ws_copies; c0 += 16) {   // sixteen loads in flight, then the zero stores
    float v[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) v[c] = c0 + c < g.ws_copies ? g.ws[(int64_t)(c0 + c) * g.ws_ld + i] : 0.f;
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      s += v[c];
      if (c0 + c < g.ws_copies) g.ws[(int64_t)(c0 + c) * g.ws_ld + i] = 0.f;
    }
  }
  float* out = i < H ? g.dgamma + i : i < 2 * H ? g.dbeta + (i - H) : i < 3 * H ? g.dq + (i - 2 * H) : g.dbias + (i - 3 * H);
  *out += s;
}

size_t fwd_smem(int H) { return (size_t)(32 + 32 * (H + 1) + 32) * sizeof(float); }
size_t bwd_smem(int H, int nw) {
  const size_t tiles = (size_t)nw * 32 * 33, red = (size_t)nw * 3 * H;
  return (size_t)(32 + 32 * (H + 1) + 32 + 32 + 64 + 2 * 32 * (H / 64) + (tiles > red ? tiles : red)) * sizeof(float);
}

size_t head_bwd_smem(int nw, int dv) { return (size_t)(64 * nw + nw * 32 * 33 + nw * 32 * (dv + 1)) * sizeof(float); }

enum Pass { FWD = 0, BWD_FUSED = 1, BWD_SPLIT = 2 };

template <typename K>
void allow_smem(K kern, size_t sz) {
  if (sz > 64 * 1024) (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sz);
}

// ---- Eval-time MHA user encoder + its pooling (MHA_User_Encoder.forward, MHA.py:58-75, over the
// per-news key / value projections the fast eval computes once per news table): per impression of
// L <= 64 history slots, per head  O_h = XSoftmax(K_h K_hᵀ / sqrt(dk), m_i m_j) V_h  (tied Q = K,
// Attention.py:125-147), then  s_l = q·O_l / sqrt(H),  p = XSoftmax(s, m),  user = Σ p_l O_l
// (Attention_Pooling, Pooling.py:12-25).  One workgroup per impression, one wave per head; the
// slots sit on 64 = 2 x 32 MFMA rows: lane (c, h) holds key rows c and c + 32 and computes the four
// 32 x 32 blocks of S from its own registers (S_{ib,jb} = K_ib K_jbᵀ: A and B are both the lane's
// rows), so it ends up holding 32 of the 64 scores of rows c and c + 32 (S is symmetric) -- the row
// softmax is in-register plus one cross-half exchange, and P feeds O = P V as the A operand
// directly (head_out's k order).  O goes to LDS [64][H + 1]; the pooling runs on it as in the
// title kernel.  Replaces mha_attn_fwd_split (scalar FMAs, 64 ms of a 14.5 M-candidate fast eval)
// + the pooling launch, and the [B N, H] attention output's HBM round trip.
template <int DK, int NP>
__device__ __forceinline__ void load_krow64(const MPArgs& g, int head, int rb, float (&a)[DK / 2]) {
  const int lane = threadIdx.x & 63, c = lane & 31, h = lane >> 5;
  const int row = c + 32 * rb;
  const bool ok = row < g.L;
  if constexpr (NP > 0) {   // a[8t + u] = K[row][16t + 8h + u]
    const float* kr = yrow(g, ok ? row : 0) + head * DK + 8 * h;
#pragma unroll
    for (int t = 0; t < DK / 16; ++t)
#pragma unroll
      for (int q4 = 0; q4 < 2; ++q4) {
        const float4 v = *reinterpret_cast<const float4*>(kr + 16 * t + 4 * q4);
        float* d = a + 8 * t + 4 * q4;
        d[0] = ok ? v.x : 0.f; d[1] = ok ? v.y : 0.f; d[2] = ok ? v.z : 0.f; d[3] = ok ? v.w : 0.f;
      }
  } else {                  // a[s + q] = K[row][4h + 2s + q]
    const float* kr = yrow(g, ok ? row : 0) + head * DK + 4 * h;
#pragma unroll
    for (int s = 0; s < DK / 2; s += 4) {
      const float4 v = *reinterpret_cast<const float4*>(kr + 2 * s);
      a[s] = ok ? v.x : 0.f; a[s + 1] = ok ? v.y : 0.f; a[s + 2] = ok ? v.z : 0.f; a[s + 3] = ok ? v.w : 0.f;
    }
  }
}

// S_{ib,jb} = K_ib K_jbᵀ over the lanes' half-rows a_i (rows of block ib) and a_j (block jb)
template <int DK, int NP>
__device__ __forceinline__ void s_block(const float (&ai)[DK / 2], const float (&aj)[DK / 2], f32x16& S) {
#pragma unroll
  for (int r = 0; r < 16; ++r) S[r] = 0.f;
  if constexpr (NP == 0) {
#pragma unroll
    for (int s = 0; s < DK / 2; ++s) S = __builtin_amdgcn_mfma_f32_32x32x2f32(ai[s], aj[s], S, 0, 0, 0);
  } else {
#pragma unroll
    for (int t = 0; t < DK / 16; ++t) mfma_x<NP>(S, planes8<NP>(ai + 8 * t), planes8<NP>(aj + 8 * t));
  }
}

// Rows c + 32 jb of one head (this lane's row of block jb): S over both key blocks, the row softmax,
// O = P V for those rows into os.  ka_j is the lane's row of block jb (ka0 or ka1).
template <int DK, int DV, int NP>
__device__ __forceinline__ void user_rows(const MPArgs& g, uint64_t bits, int head, const float (&ka0)[DK / 2],
                                          const float (&ka1)[DK / 2], const float (&ka_j)[DK / 2], int jb,
                                          const uint32_t* rw, float* os, int so) {
  const int lane = threadIdx.x & 63, c = lane & 31, h = lane >> 5;
  // p[ib][r] = P[c + 32 jb][crow(r, h) + 32 ib]
  float p[2][16];
  {
    f32x16 S0, S1;
    s_block<DK, NP>(ka0, ka_j, S0);
    s_block<DK, NP>(ka1, ka_j, S1);
    const int R = c + 32 * jb;
    const bool mr = R < g.L && ((bits >> R) & 1ull);
    float mx = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int C0 = crow(r, h), C1 = C0 + 32;
      p[0][r] = mr && ((bits >> C0) & 1ull) ? S0[r] * g.scale_attn : -INFINITY;
      p[1][r] = mr && C1 < g.L && ((bits >> C1) & 1ull) ? S1[r] * g.scale_attn : -INFINITY;
      mx = fmaxf(mx, fmaxf(p[0][r], p[1][r]));
    }
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    float sum = 0.f;
#pragma unroll
    for (int ib = 0; ib < 2; ++ib)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float e = p[ib][r] == -INFINITY ? 0.f : __expf(p[ib][r] - mx);
        p[ib][r] = e;
        sum += e;
      }
    sum += __shfl_xor(sum, 32, 64);
    const float inv = sum > 0.f ? 1.f / sum : 0.f;   // a fully masked row: zeros (XSoftmax)
#pragma unroll
    for (int ib = 0; ib < 2; ++ib)
#pragma unroll
      for (int r = 0; r < 16; ++r) p[ib][r] *= inv;
  }
  const int nq = g.heads * DK;
#pragma unroll
  for (int vb = 0; vb < DV / 32; ++vb) {
    f32x16 O;
#pragma unroll
    for (int r = 0; r < 16; ++r) O[r] = 0.f;
#pragma unroll
    for (int ib = 0; ib < 2; ++ib) {
      // V operand: bv[s] = V[crow(s, h) + 32 ib][vb * 32 + c] (slots past L: 0)
      float bv[16];
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const int k = crow(s, h) + 32 * ib;
        const float v = ld_off(g.y, rw[k < g.L ? k : 0] + 4u * (uint32_t)(nq + head * DV + vb * 32 + c));
        bv[s] = k < g.L ? v : 0.f;
      }
      mfma16<NP>(O, p[ib], bv);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = crow(r, h) + 32 * jb;
      if (row < g.L) os[row * so + head * DV + vb * 32 + c] = O[r];   // LDS holds the L real slots
    }
  }
}

template <int DK, int DV, int NH64, int NP>
__global__ __launch_bounds__(768) void mha_user_pool_fwd_kernel(MPArgs g) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  constexpr int H = NH64 * 64;
  constexpr int SO = H + 1;
  uint32_t* rw = reinterpret_cast<uint32_t*>(sm);   // [64] staged row byte offsets (yrow)
  float* os = sm + 64;                              // [L][SO]  O
  float* sc = os + g.L * SO;                        // [64] scores -> probabilities
  const int64_t seq = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, nw = blockDim.x >> 6, nt = blockDim.x;
  const int c = lane & 31, h = lane >> 5;
  const uint64_t bits = token_bits(g, seq);
  if (tid < 64) rw[tid] = row_byte_off(g, seq * g.L + (tid < g.L ? tid : 0));
  __syncthreads();
  for (int head = w; head < g.heads; head += nw) {
    float ka0[DK / 2], ka1[DK / 2];
    load_krow64<DK, NP>(g, head, 0, ka0);
    load_krow64<DK, NP>(g, head, 1, ka1);
    user_rows<DK, DV, NP>(g, bits, head, ka0, ka1, ka0, 0, rw, os, SO);
    __builtin_amdgcn_sched_barrier(0);
    user_rows<DK, DV, NP>(g, bits, head, ka0, ka1, ka1, 1, rw, os, SO);
  }
  __syncthreads();
  // pooling: s_l = q · O_l / sqrt(H), one wave per slot
  float qv[NH64];
#pragma unroll
  for (int k = 0; k < NH64; ++k) qv[k] = g.q[lane + 64 * k];
  for (int l = w; l < g.L; l += nw) {
    float dot = 0.f;
#pragma unroll
    for (int k = 0; k < NH64; ++k) dot = fmaf(qv[k], os[l * SO + lane + 64 * k], dot);
    dot = nr_wave_sum(dot);
    if (lane == 0) sc[l] = dot * g.scale_pool;
  }
  __syncthreads();
  if (w == 0) {
    const bool keep = lane < g.L && ((bits >> lane) & 1ull);
    const float v = keep ? sc[lane] : -INFINITY;
    const float mx = nr_wave_max(v);
    const float e = keep ? __expf(v - mx) : 0.f;
    const float sum = nr_wave_sum(e);
    sc[lane] = sum > 0.f ? e / sum : 0.f;
  }
  __syncthreads();
  for (int d = tid; d < H; d += nt) {
    float acc = 0.f;
    for (int l = 0; l < g.L; ++l) acc = fmaf(sc[l], os[l * SO + d], acc);
    g.news[seq * g.ldn + d] = acc;
  }
}

size_t user_pool_smem(int H, int L) { return (size_t)(64 + L * (H + 1) + 64) * sizeof(float); }
constexpr size_t NR_MAX_LDS = 160 * 1024;   // gfx950: LDS per CU, the most one workgroup may allocate

// One wave per head (twelve per impression, three per SIMD at 167 VGPRs: one workgroup per CU).  Six
// waves of two heads each, two workgroups per CU (O held for the L real slots, 77.5 KB at L = 50),
// measured 1.7x slower: predict 61 vs 35 ms (profiles/r05_q_eval_waves_ab.jsonl)
template <int DK, int DV, int NH64>
int launch_user_pool(const MPArgs& g, hipStream_t s) {
  const size_t sz = user_pool_smem(NH64 * 64, g.L);
  const int nw = g.heads < 4 ? 4 : g.heads;
  if (g.np == 3) {
    allow_smem(mha_user_pool_fwd_kernel<DK, DV, NH64, 3>, sz);
    hipLaunchKernelGGL((mha_user_pool_fwd_kernel<DK, DV, NH64, 3>), dim3((unsigned)g.nseq), dim3(64 * nw), sz, s, g);
  } else if (g.np == 1) {
    allow_smem(mha_user_pool_fwd_kernel<DK, DV, NH64, 1>, sz);
    hipLaunchKernelGGL((mha_user_pool_fwd_kernel<DK, DV, NH64, 1>), dim3((unsigned)g.nseq), dim3(64 * nw), sz, s, g);
  } else {
    allow_smem(mha_user_pool_fwd_kernel<DK, DV, NH64, 0>, sz);
    hipLaunchKernelGGL((mha_user_pool_fwd_kernel<DK, DV, NH64, 0>), dim3((unsigned)g.nseq), dim3(64 * nw), sz, s, g);
  }
  NR_LAUNCH_CHECK();
  return NR_OK;
}

template <int DK, int DV, int NH64, int NP>
int launch_np(const MPArgs& g, Pass pass, hipStream_t s) {
  const int H = NH64 * 64;
  if (pass == FWD) {
    // FOUR waves per title, each taking heads w, w + 4, ...: the workgroup's 49.5 KB LDS image then
    // lets three titles share a CU (one wave per head, 12 waves at 104 VGPRs, fit one title per CU,
    // whose barrier-separated phases left the CU idle on every load latency: 105 us per NRMS step).
    const int nw = 4;
    const size_t sz = fwd_smem(H);
    allow_smem(mha_pool_fwd_kernel<DK, DV, NH64, NP>, sz);
    hipLaunchKernelGGL((mha_pool_fwd_kernel<DK, DV, NH64, NP>), dim3((unsigned)g.nseq), dim3(64 * nw), sz, s, g);
  } else if (pass == BWD_FUSED) {
    // one wave per two heads (its per-head state needs ~200 VGPRs, more than a 12-wave
    // workgroup can give a wave); with the saved O (g.o) the O rows are loaded, not recomputed
    const int nw = (g.heads + 1) / 2 < 4 ? 4 : (g.heads + 1) / 2;
    const size_t sz = bwd_smem(H, nw);
    if (g.o) {
      allow_smem(mha_pool_bwd_kernel<DK, DV, NH64, NP, true>, sz);
      hipLaunchKernelGGL((mha_pool_bwd_kernel<DK, DV, NH64, NP, true>), dim3((unsigned)g.nseq), dim3(64 * nw), sz,
                         s, g);
    } else {
      allow_smem(mha_pool_bwd_kernel<DK, DV, NH64, NP, false>, sz);
      hipLaunchKernelGGL((mha_pool_bwd_kernel<DK, DV, NH64, NP, false>), dim3((unsigned)g.nseq), dim3(64 * nw), sz,
                         s, g);
    }
    if (g.ws) {
      const int NY = g.heads * (DK + DV);
      hipLaunchKernelGGL(copies_reduce_kernel, dim3((unsigned)((3 * H + NY + 63) / 64)), dim3(64), 0, s, g, H, NY);
    }
  } else {
    hipLaunchKernelGGL((mha_ln_bwd_kernel<NH64>), dim3((unsigned)g.nseq), dim3(256), 0, s, g);
    MPArgs g2 = g;
    g2.rows_per_wave = 1;
    const unsigned gx = (unsigned)((g.nseq + HB_TITLES - 1) / HB_TITLES), gy = (unsigned)((g.heads + 3) / 4);
    hipLaunchKernelGGL((mha_head_bwd_kernel<DK, DV, NP>), dim3(gx, gy), dim3(256), head_bwd_smem(4, DV), s, g2);
    if (g.ws) {
      const int NY = g.heads * (DK + DV);
      hipLaunchKernelGGL(copies_reduce_kernel, dim3((unsigned)((3 * H + NY + 63) / 64)), dim3(64), 0, s, g, H, NY);
    }
  }
  NR_LAUNCH_CHECK();
  return NR_OK;
}

// the attention products' arithmetic follows the caller's GEMM precision (nr_gemm_precision)
template <int DK, int DV, int NH64>
int launch(const MPArgs& g, Pass pass, hipStream_t s) {
  if (g.np == 3) return launch_np<DK, DV, NH64, 3>(g, pass, s);
  if (g.np == 1) return launch_np<DK, DV, NH64, 1>(g, pass, s);
  return launch_np<DK, DV, NH64, 0>(g, pass, s);
}

int dispatch(const MPArgs& g, int dk, int dv, Pass pass, hipStream_t s) {
  const int H = g.heads * dv;
  if (H % 64) return NR_EINVAL(9);
  const int nh64 = H / 64;
#define NR_CASE(K, V, N) \
  if (dk == K && dv == V && nh64 == N) return launch<K, V, N>(g, pass, s);
  NR_CASE(64, 32, 6)    // NRMS news encoder: E=768 -> 12 heads x 64, H = 384
  NR_CASE(64, 64, 12)   // H = 768
  NR_CASE(64, 32, 4)    // H = 256 (8 heads)
  NR_CASE(32, 32, 6)
#undef NR_CASE
  return NR_EINVAL(8);
}

bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

extern "C" int nr_mha_pool_fwd(const float* y, int64_t ldy, const int64_t* yrows, const void* mask,
                               int32_t mask_dtype, int64_t nseq,
                               int32_t L, int32_t heads, int32_t dk, int32_t dv, const float* gamma,
                               const float* beta, float eps, float p_drop, uint64_t seed, uint64_t offset, const uint64_t* rng,
                               const float* q, float* news, int64_t ldn, float* zout, int64_t ldz, float* oout,
                               int64_t ldo, float* stats, float* probs, int32_t prec, hipStream_t stream) {
  if (L < 1 || L > 32 || heads < 1 || heads > 12) return NR_EINVAL(0);
  if (prec != NR_GEMM_F32 && prec != NR_GEMM_BF16X6 && prec != NR_GEMM_BF16) return NR_EINVAL(4);
  if (!y || !mask || !gamma || !beta || !q || !news || !stats || !probs) return NR_EINVAL(1);
  if ((ldy & 3) || !al16(y)) return NR_EINVAL(2);
  if (nseq == 0) return NR_OK;
  MPArgs g{};
  g.y = y; g.ldy = ldy; g.yrows = yrows; g.mask = mask; g.mask_dt = mask_dtype; g.nseq = nseq; g.L = L; g.heads = heads;
  g.scale_attn = 1.0f / sqrtf((float)dk); g.scale_pool = 1.0f / sqrtf((float)(heads * dv));
  g.gamma = gamma; g.beta = beta; g.eps = eps; g.p_drop = p_drop; g.seed = seed; g.offset = offset;
  g.dkey = nr_dropout_key(seed, offset); g.dthresh = nr_dropout_threshold(p_drop); g.rng = rng; g.q = q;
  g.news = news; g.ldn = ldn; g.zout = zout; g.ldz = ldz; g.stats = stats; g.probs = probs;
  g.o = oout; g.ldo = ldo;
  if (oout && ((ldo & 3) || ldo < (int64_t)heads * dv)) return NR_EINVAL(3);
  g.np = prec == NR_GEMM_BF16X6 ? 3 : prec == NR_GEMM_BF16 ? 1 : 0;
  return dispatch(g, dk, dv, FWD, stream);
}

extern "C" int nr_mha_user_pool_fwd(const float* y, int64_t ldy, int64_t y_rows, const int64_t* yrows,
                                    const void* mask, int32_t mask_dtype, int64_t nseq, int32_t L, int32_t heads,
                                    int32_t dk, int32_t dv, const float* q, float* out, int64_t ldo, int32_t prec,
                                    hipStream_t stream) {
  if (L < 1 || L > 64 || heads < 1 || heads > 12) return NR_EINVAL(0);
  if (y_rows < 1 || y_rows * ldy * 4 >= ((int64_t)1 << 32)) return NR_EINVAL(5);   // 32-bit row byte offsets
  if (prec != NR_GEMM_F32 && prec != NR_GEMM_BF16X6 && prec != NR_GEMM_BF16) return NR_EINVAL(4);
  if (!y || !mask || !q || !out) return NR_EINVAL(1);
  if ((ldy & 3) || !al16(y) || ldy < (int64_t)heads * (dk + dv)) return NR_EINVAL(2);
  if (ldo < (int64_t)heads * dv) return NR_EINVAL(3);
  if (nseq == 0) return NR_OK;
  MPArgs g{};
  g.y = y; g.ldy = ldy; g.yrows = yrows; g.mask = mask; g.mask_dt = mask_dtype; g.nseq = nseq; g.L = L;
  g.heads = heads; g.scale_attn = 1.0f / sqrtf((float)dk); g.scale_pool = 1.0f / sqrtf((float)(heads * dv));
  g.q = q; g.news = out; g.ldn = ldo;
  g.np = prec == NR_GEMM_BF16X6 ? 3 : prec == NR_GEMM_BF16 ? 1 : 0;
  const int nh64 = heads * dv / 64;
  if ((heads * dv) % 64) return NR_EINVAL(9);
  // O [L][H + 1] stays in LDS: at H = 768 that caps L at 53 (the caller falls back to the two-launch
  // path, kernels.mha_user_pool_supported)
  if (user_pool_smem(heads * dv, L) > NR_MAX_LDS) return NR_EINVAL(10);
  if (dk == 32 && dv == 32 && nh64 == 6) return launch_user_pool<32, 32, 6>(g, stream);
  if (dk == 64 && dv == 32 && nh64 == 6) return launch_user_pool<64, 32, 6>(g, stream);
  if (dk == 64 && dv == 64 && nh64 == 12) return launch_user_pool<64, 64, 12>(g, stream);
  return NR_EINVAL(8);
}

extern "C" int nr_mha_pool_bwd(const float* y, int64_t ldy, const int64_t* yrows, const void* mask,
                               int32_t mask_dtype, int64_t nseq,
                               int32_t L, int32_t heads, int32_t dk, int32_t dv, const float* gamma,
                               const float* beta, float p_drop, uint64_t seed, uint64_t offset, const uint64_t* rng, const float* q,
                               const float* stats, const float* probs, const float* dnews, int64_t ldn,
                               const float* dz, int64_t lddz, const float* o, int64_t ldo, float* dob,
                               int64_t lddob, float* dy, int64_t lddy, float* dbias, float* dq, float* dgamma,
                               float* dbeta, float* ws, int32_t ws_copies, const int32_t* seg_off,
                               int64_t dyu_row0, int64_t dy_rows, uint32_t* dsto, int32_t prec, hipStream_t stream) {
  if (L < 1 || L > 32 || heads < 1 || heads > 12) return NR_EINVAL(0);
  if (prec != NR_GEMM_F32 && prec != NR_GEMM_BF16X6 && prec != NR_GEMM_BF16) return NR_EINVAL(4);
  if (!y || !mask || !gamma || !beta || !q || !stats || !probs || !dnews || !dy || !dbias || !dq || !dgamma ||
      !dbeta)
    return NR_EINVAL(1);
  // dy rows addressed by 32-bit byte offsets from dy
  if (dy_rows < nseq * L || dy_rows * lddy * 4 >= ((int64_t)1 << 32)) return NR_EINVAL(6);
  if (seg_off && (!yrows || !dsto || dyu_row0 < nseq * L || dyu_row0 > dy_rows)) return NR_EINVAL(7);
  if ((ldy & 3) || !al16(y)) return NR_EINVAL(2);
  if (nseq == 0) return NR_OK;
  MPArgs g{};
  g.y = y; g.ldy = ldy; g.yrows = yrows; g.mask = mask; g.mask_dt = mask_dtype; g.nseq = nseq; g.L = L; g.heads = heads;
  g.scale_attn = 1.0f / sqrtf((float)dk); g.scale_pool = 1.0f / sqrtf((float)(heads * dv));
  g.gamma = gamma; g.beta = beta; g.p_drop = p_drop; g.seed = seed; g.offset = offset;
  g.dkey = nr_dropout_key(seed, offset); g.dthresh = nr_dropout_threshold(p_drop); g.rng = rng; g.q = q;
  g.news = const_cast<float*>(dnews); g.ldn = ldn; g.stats = const_cast<float*>(stats);
  g.probs = const_cast<float*>(probs); g.dz = dz; g.lddz = lddz; g.dy = dy; g.lddy = lddy; g.dbias = dbias;
  g.dq = dq; g.dgamma = dgamma; g.dbeta = dbeta;
  g.o = const_cast<float*>(o); g.ldo = ldo; g.dob = dob; g.lddob = lddob;
  g.seg_off = seg_off; g.dyu_row0 = dyu_row0; g.dsto = seg_off ? dsto : nullptr;
  // o with dob: the split backward (dob: the LN pass's per-token row terms, [T][>= 8] floats); o without
  // dob: the fused backward on the saved O
  if (o && ((dob && (lddob < 8 || (lddob & 3) || !al16(dob))) || ldo < (int64_t)heads * dv || (ldo & 3) || !al16(o)))
    return NR_EINVAL(3);
  // backward: the six-product form measured slower than exact f32 MFMA products here (the split
  // VALU work lands on a latency-bound kernel: head pass 170 -> 189 us), so bf16x6 callers get the
  // exact (more accurate) f32 products; bf16 callers get bf16
  g.np = prec == NR_GEMM_BF16 ? 1 : 0;
  if (ws && (!o || ws_copies < 1 || ws_copies > 1024)) return NR_EINVAL(5);
  g.ws = ws; g.ws_copies = ws_copies;
  g.ws_ld = ((int64_t)3 * heads * dv + (int64_t)heads * (dk + dv) + 3) & ~int64_t(3);
  return dispatch(g, dk, dv, o && dob ? BWD_SPLIT : BWD_FUSED, stream);
}
