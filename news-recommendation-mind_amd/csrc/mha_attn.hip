// Small-sequence multi-head self attention with TIED query/key projections, the reference's
// MultiheadAttention core (models/Modules/Attention.py:115-147):
//     S_h = Kp_h Kp_hᵀ / sqrt(d_k)            (Q and K are both keyProject(x), :125-126)
//     P_h = XSoftmax(S_h, m_i * m_j)           (:56-80, get_attn_mask :33-53)
//     O_h = P_h Vp_h, heads concatenated        (no output projection)
// Sequences are short (news titles L = 30, click histories N = 50), so one wave owns one
// (sequence, head) — or two heads when L <= 32 — with one ROW PER LANE: the lane keeps its
// query row and its score row in registers, the head's K/V rows sit in LDS and are read as
// wave-uniform broadcasts.  Masked slots get probability exactly 0 and a fully masked row is
// all-zero (XSoftmax's masked_fill after softmax), never NaN.
//
// Backward recomputes P from Kp (nothing but the inputs is saved) and produces
//   dV_j = Σ_i P_ij dO_i,  dS = P ∘ (dP − rowsum(P ∘ dP)),  dP_ij = dO_i · V_j,
//   dKp_i = scale · Σ_j (dS_ij + dS_ji) Kp_j          (Kp feeds both the Q and the K role).
#include "common.h"
#include "../../include/newsrec_hip.h"

namespace {

struct AttnArgs {
  const float* qk; int64_t ld_qk;
  const float* v; int64_t ld_v;
  const void* mask; int mask_dt;
  int64_t nseq; int L; int heads; float scale;
  const float* dout; int64_t ld_dout;   // bwd: dO
  float* out; int64_t ld_out;           // fwd: O         bwd: dKp
  float* dv; int64_t ld_dv;             // bwd: dVp
  const int64_t* rows;                  // fwd: physical qk / v row of token (seq*L + j), or null
};

template <int LMAX, int DK, int DV>
struct Smem {
  static constexpr int HPW = 64 / LMAX;          // heads per wave
  float k[HPW][LMAX][DK];
  float v[HPW][LMAX][DV];
  float p[HPW][LMAX][LMAX + 1];                  // P then dS (bwd)
  float d[HPW][LMAX][DV];                        // dO (bwd)
};

// forward: K/V rows only (16 KB at L <= 64, dk = dv = 32 instead of 41 KB: 2.5x the resident
// waves per CU)
template <int LMAX, int DK, int DV>
struct SmemF {
  static constexpr int HPW = 64 / LMAX;
  float k[HPW][LMAX][DK];
  float v[HPW][LMAX][DV];
};

template <bool WITH_DOUT, int LMAX, int DK, int DV, class S>
__device__ __forceinline__ void load_rows(S& sm, const AttnArgs& g, int64_t seq, int head0) {
  constexpr int HPW = 64 / LMAX;
  const int lane = threadIdx.x;
  // K rows: HPW heads x L rows x DK floats, as float4
  constexpr int K4 = DK / 4, V4 = DV / 4;
  for (int e = lane; e < HPW * LMAX * K4; e += 64) {
    const int hh = e / (LMAX * K4), rem = e % (LMAX * K4), j = rem / K4, c = rem % K4;
    float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
    if (j < g.L && head0 + hh < g.heads) {
      const int64_t r = g.rows ? g.rows[seq * g.L + j] : seq * g.L + j;
      x = *reinterpret_cast<const float4*>(g.qk + r * g.ld_qk + (head0 + hh) * DK + 4 * c);
    }
    *reinterpret_cast<float4*>(&sm.k[hh][j][4 * c]) = x;
  }
  for (int e = lane; e < HPW * LMAX * V4; e += 64) {
    const int hh = e / (LMAX * V4), rem = e % (LMAX * V4), j = rem / V4, c = rem % V4;
    float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 y = x;
    if (j < g.L && head0 + hh < g.heads) {
      const int64_t r = g.rows ? g.rows[seq * g.L + j] : seq * g.L + j;
      x = *reinterpret_cast<const float4*>(g.v + r * g.ld_v + (head0 + hh) * DV + 4 * c);
      if constexpr (WITH_DOUT)
        y = *reinterpret_cast<const float4*>(g.dout + (seq * g.L + j) * g.ld_dout + (head0 + hh) * DV + 4 * c);
    }
    *reinterpret_cast<float4*>(&sm.v[hh][j][4 * c]) = x;
    if constexpr (WITH_DOUT) *reinterpret_cast<float4*>(&sm.d[hh][j][4 * c]) = y;
  }
}

// Row i of P for the lane's head: returns probabilities in p[], exact zeros where masked.
template <int LMAX, int DK, int DV, class S>
__device__ __forceinline__ void softmax_row(const S& sm, const AttnArgs& g,
                                            int64_t seq, int hh, int i, bool row_ok, float (&q)[DK],
                                            float (&p)[LMAX]) {
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < LMAX; ++j) {
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < DK; c += 4) {
      const float4 kj = *reinterpret_cast<const float4*>(&sm.k[hh][j][c]);
      s = fmaf(q[c], kj.x, s); s = fmaf(q[c + 1], kj.y, s);
      s = fmaf(q[c + 2], kj.z, s); s = fmaf(q[c + 3], kj.w, s);
    }
    const bool keep = row_ok && j < g.L && nr_mask_at(g.mask, g.mask_dt, seq * g.L + j);
    p[j] = keep ? s * g.scale : -INFINITY;
    mx = fmaxf(mx, p[j]);
  }
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < LMAX; ++j) {
    const float e = p[j] == -INFINITY ? 0.f : __expf(p[j] - mx);
    p[j] = e;
    sum += e;
  }
  const float inv = sum > 0.f ? 1.f / sum : 0.f;
#pragma unroll
  for (int j = 0; j < LMAX; ++j) p[j] *= inv;
}

template <int LMAX, int DK, int DV>
__global__ __launch_bounds__(64) void mha_attn_fwd_kernel(AttnArgs g) {
  constexpr int HPW = 64 / LMAX;
  __shared__ __attribute__((aligned(16))) SmemF<LMAX, DK, DV> sm;
  const int64_t seq = blockIdx.x;
  const int head0 = blockIdx.y * HPW;
  const int lane = threadIdx.x, hh = lane / LMAX, i = lane % LMAX;
  const int head = head0 + hh;
  load_rows<false, LMAX, DK, DV>(sm, g, seq, head0);
  __syncthreads();
  if (head >= g.heads || i >= g.L) return;
  const bool row_ok = nr_mask_at(g.mask, g.mask_dt, seq * g.L + i);
  float q[DK];
#pragma unroll
  for (int c = 0; c < DK; ++c) q[c] = sm.k[hh][i][c];
  float p[LMAX];
  softmax_row<LMAX, DK, DV>(sm, g, seq, hh, i, row_ok, q, p);
  float o[DV];
#pragma unroll
  for (int c = 0; c < DV; ++c) o[c] = 0.f;
#pragma unroll
  for (int j = 0; j < LMAX; ++j) {
#pragma unroll
    for (int c = 0; c < DV; c += 4) {
      const float4 vj = *reinterpret_cast<const float4*>(&sm.v[hh][j][c]);
      o[c] = fmaf(p[j], vj.x, o[c]); o[c + 1] = fmaf(p[j], vj.y, o[c + 1]);
      o[c + 2] = fmaf(p[j], vj.z, o[c + 2]); o[c + 3] = fmaf(p[j], vj.w, o[c + 3]);
    }
  }
  float* dst = g.out + (seq * g.L + i) * g.ld_out + head * DV;
#pragma unroll
  for (int c = 0; c < DV; c += 4)
    *reinterpret_cast<float4*>(dst + c) = make_float4(o[c], o[c + 1], o[c + 2], o[c + 3]);
}

template <int LMAX, int DK, int DV>
__global__ __launch_bounds__(64) void mha_attn_bwd_kernel(AttnArgs g) {
  constexpr int HPW = 64 / LMAX;
  __shared__ __attribute__((aligned(16))) Smem<LMAX, DK, DV> sm;
  const int64_t seq = blockIdx.x;
  const int head0 = blockIdx.y * HPW;
  const int lane = threadIdx.x, hh = lane / LMAX, i = lane % LMAX;
  const int head = head0 + hh;
  load_rows<true, LMAX, DK, DV>(sm, g, seq, head0);
  __syncthreads();
  const bool active = head < g.heads && i < g.L;
  const bool row_ok = active && nr_mask_at(g.mask, g.mask_dt, seq * g.L + i);

  float q[DK];
#pragma unroll
  for (int c = 0; c < DK; ++c) q[c] = sm.k[hh][i][c];
  float p[LMAX];
  softmax_row<LMAX, DK, DV>(sm, g, seq, hh, i, row_ok, q, p);
  // P row -> LDS (dV needs P columns)
#pragma unroll
  for (int j = 0; j < LMAX; ++j) sm.p[hh][i][j] = p[j];
  // dP_ij = dO_i . V_j ; rowsum(P ∘ dP)
  float dO[DV];
#pragma unroll
  for (int c = 0; c < DV; ++c) dO[c] = sm.d[hh][i][c];
  float dp[LMAX];
  float rs = 0.f;
#pragma unroll
  for (int j = 0; j < LMAX; ++j) {
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < DV; c += 4) {
      const float4 vj = *reinterpret_cast<const float4*>(&sm.v[hh][j][c]);
      s = fmaf(dO[c], vj.x, s); s = fmaf(dO[c + 1], vj.y, s);
      s = fmaf(dO[c + 2], vj.z, s); s = fmaf(dO[c + 3], vj.w, s);
    }
    dp[j] = s;
    rs = fmaf(p[j], s, rs);
  }
  __syncthreads();
  // dV_i (this lane's row as the KEY index) = Σ_r P_ri dO_r
  {
    float acc[DV];
#pragma unroll
    for (int c = 0; c < DV; ++c) acc[c] = 0.f;
#pragma unroll
    for (int r = 0; r < LMAX; ++r) {
      const float pr = sm.p[hh][r][i];
#pragma unroll
      for (int c = 0; c < DV; c += 4) {
        const float4 d4 = *reinterpret_cast<const float4*>(&sm.d[hh][r][c]);
        acc[c] = fmaf(pr, d4.x, acc[c]); acc[c + 1] = fmaf(pr, d4.y, acc[c + 1]);
        acc[c + 2] = fmaf(pr, d4.z, acc[c + 2]); acc[c + 3] = fmaf(pr, d4.w, acc[c + 3]);
      }
    }
    if (active) {
      float* dst = g.dv + (seq * g.L + i) * g.ld_dv + head * DV;
#pragma unroll
      for (int c = 0; c < DV; c += 4)
        *reinterpret_cast<float4*>(dst + c) = make_float4(acc[c], acc[c + 1], acc[c + 2], acc[c + 3]);
    }
  }
  __syncthreads();
  // dS row (scaled) overwrites P in LDS
#pragma unroll
  for (int j = 0; j < LMAX; ++j) sm.p[hh][i][j] = p[j] * (dp[j] - rs) * g.scale;
  __syncthreads();
  if (!active) return;
  float acc[DK];
#pragma unroll
  for (int c = 0; c < DK; ++c) acc[c] = 0.f;
#pragma unroll
  for (int j = 0; j < LMAX; ++j) {
    const float w = sm.p[hh][i][j] + sm.p[hh][j][i];
#pragma unroll
    for (int c = 0; c < DK; c += 4) {
      const float4 kj = *reinterpret_cast<const float4*>(&sm.k[hh][j][c]);
      acc[c] = fmaf(w, kj.x, acc[c]); acc[c + 1] = fmaf(w, kj.y, acc[c + 1]);
      acc[c + 2] = fmaf(w, kj.z, acc[c + 2]); acc[c + 3] = fmaf(w, kj.w, acc[c + 3]);
    }
  }
  float* dst = g.out + (seq * g.L + i) * g.ld_out + head * DK;
#pragma unroll
  for (int c = 0; c < DK; c += 4)
    *reinterpret_cast<float4*>(dst + c) = make_float4(acc[c], acc[c + 1], acc[c + 2], acc[c + 3]);
}

template <int LMAX, int DK, int DV>
int launch(const AttnArgs& g, bool bwd, hipStream_t s) {
  constexpr int HPW = 64 / LMAX;
  dim3 grid((unsigned)g.nseq, (unsigned)((g.heads + HPW - 1) / HPW));
  if (bwd)
    hipLaunchKernelGGL((mha_attn_bwd_kernel<LMAX, DK, DV>), grid, dim3(64), 0, s, g);
  else
    hipLaunchKernelGGL((mha_attn_fwd_kernel<LMAX, DK, DV>), grid, dim3(64), 0, s, g);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

int dispatch(const AttnArgs& g, int dk, int dv, bool bwd, hipStream_t s) {
  const int lmax = g.L <= 32 ? 32 : 64;
#define NR_CASE(LM, K, V) \
  if (lmax == LM && dk == K && dv == V) return launch<LM, K, V>(g, bwd, s);
  NR_CASE(32, 64, 32) NR_CASE(32, 32, 32) NR_CASE(32, 64, 64) NR_CASE(32, 64, 16)
  NR_CASE(64, 32, 32) NR_CASE(64, 64, 64) NR_CASE(64, 16, 16) NR_CASE(64, 64, 32)
  NR_CASE(32, 16, 16)
#undef NR_CASE
  return NR_EINVAL(8);
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

extern "C" int nr_mha_attn_fwd(const float* qk, int64_t ld_qk, const float* v, int64_t ld_v,
                               const int64_t* rows, const void* mask, int32_t mask_dtype, int64_t nseq, int32_t L,
                               int32_t heads, int32_t dk, int32_t dv, float scale, float* out,
                               int64_t ld_out, hipStream_t stream) {
  if (L < 1 || L > 64 || heads < 1) return NR_EINVAL(0);
  if (!qk || !v || !mask || !out) return NR_EINVAL(1);
  if ((ld_qk | ld_v | ld_out) & 3 || !aligned16(qk) || !aligned16(v) || !aligned16(out)) return NR_EINVAL(2);
  if (nseq == 0) return NR_OK;
  AttnArgs g{qk, ld_qk, v, ld_v, mask, mask_dtype, nseq, L, heads, scale,
             nullptr, 0, out, ld_out, nullptr, 0, rows};
  return dispatch(g, dk, dv, false, stream);
}

extern "C" int nr_mha_attn_bwd(const float* qk, int64_t ld_qk, const float* v, int64_t ld_v,
                               const void* mask, int32_t mask_dtype, int64_t nseq, int32_t L,
                               int32_t heads, int32_t dk, int32_t dv, float scale,
                               const float* dout, int64_t ld_dout, float* dqk, int64_t ld_dqk,
                               float* dvout, int64_t ld_dv, hipStream_t stream) {
  if (L < 1 || L > 64 || heads < 1) return NR_EINVAL(0);
  if (!qk || !v || !mask || !dout || !dqk || !dvout) return NR_EINVAL(1);
  if ((ld_qk | ld_v | ld_dout | ld_dqk | ld_dv) & 3 || !aligned16(qk) || !aligned16(v) ||
      !aligned16(dout) || !aligned16(dqk) || !aligned16(dvout))
    return NR_EINVAL(2);
  if (nseq == 0) return NR_OK;
  AttnArgs g{qk, ld_qk, v, ld_v, mask, mask_dtype, nseq, L, heads, scale,
             dout, ld_dout, dqk, ld_dqk, dvout, ld_dv, nullptr};
  return dispatch(g, dk, dv, true, stream);
}
