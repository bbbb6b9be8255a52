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
// bits: the sequence's token mask (bit j = token j kept), read once per wave -- a mask load per key
// inside the loop was a serialised scalar load per score
__device__ __forceinline__ uint64_t seq_mask_bits(const AttnArgs& g, int64_t seq) {
  const int lane = threadIdx.x & 63;
  return __ballot(lane < g.L && nr_mask_at(g.mask, g.mask_dt, seq * g.L + lane));
}

template <int LMAX, int DK, int DV, class S>
__device__ __forceinline__ void softmax_row(const S& sm, const AttnArgs& g, uint64_t bits, int hh, bool row_ok,
                                            float (&q)[DK], float (&p)[LMAX]) {
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
    const bool keep = row_ok && ((bits >> j) & 1ull);
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
  const uint64_t bits = seq_mask_bits(g, seq);
  load_rows<false, LMAX, DK, DV>(sm, g, seq, head0);
  __syncthreads();
  if (head >= g.heads || i >= g.L) return;
  const bool row_ok = (bits >> i) & 1ull;
  float q[DK];
#pragma unroll
  for (int c = 0; c < DK; ++c) q[c] = sm.k[hh][i][c];
  float p[LMAX];
  softmax_row<LMAX, DK, DV>(sm, g, bits, hh, row_ok, q, p);
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
  const uint64_t bits = seq_mask_bits(g, seq);
  load_rows<true, LMAX, DK, DV>(sm, g, seq, head0);
  __syncthreads();
  const bool active = head < g.heads && i < g.L;
  const bool row_ok = active && ((bits >> i) & 1ull);

  float q[DK];
#pragma unroll
  for (int c = 0; c < DK; ++c) q[c] = sm.k[hh][i][c];
  float p[LMAX];
  softmax_row<LMAX, DK, DV>(sm, g, bits, hh, row_ok, q, p);
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

// ---- L in (32, 64] (the user encoder's 50-click histories: few sequences): FOUR waves per
// (sequence, head), rows on the lanes as above, the key loops split over the waves -- a wave's
// serial instruction stream is a quarter as long.  Forward: each wave takes 16 keys, keeps a
// partial (max, sum, P·V) per row, and the partials are merged through LDS (online-softmax
// rescaling).  Backward: scores and dP over the wave's 16 keys (row max / sum / rowsum(P∘dP) merged
// through LDS), then dV and dK with the wave owning a quarter of the feature columns.
constexpr int SPLIT_NW = 4;

template <bool WITH_DOUT, int DK, int DV>
__device__ __forceinline__ void load_rows_split(const AttnArgs& g, int64_t seq, int head, float (*k)[DK],
                                                float (*v)[DV], float (*d)[DV]) {
  constexpr int K4 = DK / 4, V4 = DV / 4;
  for (int e = threadIdx.x; e < 64 * (K4 + V4); e += 64 * SPLIT_NW) {
    const bool isk = e < 64 * K4;
    const int e2 = isk ? e : e - 64 * K4, W4 = isk ? K4 : V4;
    const int j = e2 / W4, c = e2 % W4;
    float4 x = make_float4(0.f, 0.f, 0.f, 0.f), y = x;
    if (j < g.L) {
      const int64_t r = g.rows ? g.rows[seq * g.L + j] : seq * g.L + j;
      if (isk) {
        x = *reinterpret_cast<const float4*>(g.qk + r * g.ld_qk + head * DK + 4 * c);
      } else {
        x = *reinterpret_cast<const float4*>(g.v + r * g.ld_v + head * DV + 4 * c);
        if constexpr (WITH_DOUT)
          y = *reinterpret_cast<const float4*>(g.dout + (seq * g.L + j) * g.ld_dout + head * DV + 4 * c);
      }
    }
    if (isk) {
      *reinterpret_cast<float4*>(&k[j][4 * c]) = x;
    } else {
      *reinterpret_cast<float4*>(&v[j][4 * c]) = x;
      if constexpr (WITH_DOUT) *reinterpret_cast<float4*>(&d[j][4 * c]) = y;
    }
  }
}

// scores of row i against the wave's 16 keys (scaled; -inf where masked); returns the wave-local max
template <int DK>
__device__ __forceinline__ float split_scores(const float (*k)[DK], const float (&q)[DK], uint64_t bits, bool row_ok,
                                              float scale, int w, float (&s)[64 / SPLIT_NW]) {
  constexpr int JW = 64 / SPLIT_NW;
  float mx = -INFINITY;
#pragma unroll
  for (int jj = 0; jj < JW; ++jj) {
    const int j = w * JW + jj;
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int c = 0; c < DK; c += 4) {
      const float4 kj = *reinterpret_cast<const float4*>(&k[j][c]);
      a = fmaf(q[c], kj.x, a); b = fmaf(q[c + 1], kj.y, b);
      a = fmaf(q[c + 2], kj.z, a); b = fmaf(q[c + 3], kj.w, b);
    }
    const bool keep = row_ok && ((bits >> j) & 1ull);
    s[jj] = keep ? (a + b) * scale : -INFINITY;
    mx = fmaxf(mx, s[jj]);
  }
  return mx;
}

template <int DK, int DV>
__global__ __launch_bounds__(64 * SPLIT_NW) void mha_attn_fwd_split_kernel(AttnArgs g) {
  constexpr int JW = 64 / SPLIT_NW, CW = DV / SPLIT_NW;
  __shared__ __attribute__((aligned(16))) float k[64][DK];
  __shared__ __attribute__((aligned(16))) float v[64][DV];
  __shared__ float mrow[SPLIT_NW][64], lrow[SPLIT_NW][64];
  __shared__ float opart[SPLIT_NW][64][DV + 1];
  const int64_t seq = blockIdx.x;
  const int head = blockIdx.y;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, i = lane;
  const uint64_t bits = seq_mask_bits(g, seq);
  load_rows_split<false, DK, DV>(g, seq, head, k, v, nullptr);
  __syncthreads();
  const bool row_ok = (bits >> i) & 1ull;
  float q[DK];
#pragma unroll
  for (int c = 0; c < DK; ++c) q[c] = k[i][c];
  float s[JW];
  const float m = split_scores<DK>(k, q, bits, row_ok, g.scale, w, s);
  float l = 0.f, o[DV];
#pragma unroll
  for (int c = 0; c < DV; ++c) o[c] = 0.f;
#pragma unroll
  for (int jj = 0; jj < JW; ++jj) {
    const float e = s[jj] == -INFINITY ? 0.f : __expf(s[jj] - m);
    l += e;
    const int j = w * JW + jj;
#pragma unroll
    for (int c = 0; c < DV; c += 4) {
      const float4 vj = *reinterpret_cast<const float4*>(&v[j][c]);
      o[c] = fmaf(e, vj.x, o[c]); o[c + 1] = fmaf(e, vj.y, o[c + 1]);
      o[c + 2] = fmaf(e, vj.z, o[c + 2]); o[c + 3] = fmaf(e, vj.w, o[c + 3]);
    }
  }
  mrow[w][i] = m;
  lrow[w][i] = l;
#pragma unroll
  for (int c = 0; c < DV; ++c) opart[w][i][c] = o[c];
  __syncthreads();
  if (i >= g.L) return;
  // merge: row i, this wave's CW output columns
  float M = -INFINITY;
#pragma unroll
  for (int ww = 0; ww < SPLIT_NW; ++ww) M = fmaxf(M, mrow[ww][i]);
  float f[SPLIT_NW], Ls = 0.f;
#pragma unroll
  for (int ww = 0; ww < SPLIT_NW; ++ww) {
    f[ww] = mrow[ww][i] == -INFINITY ? 0.f : __expf(mrow[ww][i] - M);
    Ls = fmaf(lrow[ww][i], f[ww], Ls);
  }
  const float inv = Ls > 0.f ? 1.f / Ls : 0.f;   // fully masked row: zeros (XSoftmax)
  float* dst = g.out + (seq * g.L + i) * g.ld_out + head * DV + w * CW;
#pragma unroll
  for (int c = 0; c < CW; c += 4) {
    float r[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float a = 0.f;
#pragma unroll
      for (int ww = 0; ww < SPLIT_NW; ++ww) a = fmaf(opart[ww][i][w * CW + c + u], f[ww], a);
      r[u] = a * inv;
    }
    *reinterpret_cast<float4*>(dst + c) = make_float4(r[0], r[1], r[2], r[3]);
  }
}

template <int DK, int DV>
__global__ __launch_bounds__(64 * SPLIT_NW) void mha_attn_bwd_split_kernel(AttnArgs g) {
  constexpr int JW = 64 / SPLIT_NW, CK = DK / SPLIT_NW, CV = DV / SPLIT_NW;
  __shared__ __attribute__((aligned(16))) float k[64][DK];
  __shared__ __attribute__((aligned(16))) float v[64][DV];
  __shared__ __attribute__((aligned(16))) float d[64][DV];
  __shared__ float pm[64][65];   // P
  __shared__ float ds[64][65];   // dS (scaled)
  __shared__ float mrow[SPLIT_NW][64], lrow[SPLIT_NW][64], rrow[SPLIT_NW][64];
  const int64_t seq = blockIdx.x;
  const int head = blockIdx.y;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, i = lane;
  const uint64_t bits = seq_mask_bits(g, seq);
  load_rows_split<true, DK, DV>(g, seq, head, k, v, d);
  __syncthreads();
  const bool row_ok = (bits >> i) & 1ull;
  // (1) scores over the wave's keys, row max / sum merged through LDS -> P
  float q[DK];
#pragma unroll
  for (int c = 0; c < DK; ++c) q[c] = k[i][c];
  float s[JW];
  const float m = split_scores<DK>(k, q, bits, row_ok, g.scale, w, s);
  float l = 0.f;
#pragma unroll
  for (int jj = 0; jj < JW; ++jj) l += s[jj] == -INFINITY ? 0.f : __expf(s[jj] - m);
  mrow[w][i] = m;
  lrow[w][i] = l;
  __syncthreads();
  float M = -INFINITY, Ls = 0.f;
#pragma unroll
  for (int ww = 0; ww < SPLIT_NW; ++ww) M = fmaxf(M, mrow[ww][i]);
#pragma unroll
  for (int ww = 0; ww < SPLIT_NW; ++ww)
    Ls += mrow[ww][i] == -INFINITY ? 0.f : lrow[ww][i] * __expf(mrow[ww][i] - M);
  const float inv = Ls > 0.f ? 1.f / Ls : 0.f;
  // (2) dP over the wave's keys, rowsum(P ∘ dP) merged through LDS
  float dO[DV];
#pragma unroll
  for (int c = 0; c < DV; ++c) dO[c] = d[i][c];
  float p[JW], dp[JW], rs = 0.f;
#pragma unroll
  for (int jj = 0; jj < JW; ++jj) {
    const int j = w * JW + jj;
    p[jj] = s[jj] == -INFINITY ? 0.f : __expf(s[jj] - M) * inv;
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int c = 0; c < DV; c += 4) {
      const float4 vj = *reinterpret_cast<const float4*>(&v[j][c]);
      a = fmaf(dO[c], vj.x, a); b = fmaf(dO[c + 1], vj.y, b);
      a = fmaf(dO[c + 2], vj.z, a); b = fmaf(dO[c + 3], vj.w, b);
    }
    dp[jj] = a + b;
    rs = fmaf(p[jj], dp[jj], rs);
    pm[i][j] = p[jj];
  }
  rrow[w][i] = rs;
  __syncthreads();
  float R = 0.f;
#pragma unroll
  for (int ww = 0; ww < SPLIT_NW; ++ww) R += rrow[ww][i];
#pragma unroll
  for (int jj = 0; jj < JW; ++jj) ds[i][w * JW + jj] = p[jj] * (dp[jj] - R) * g.scale;
  __syncthreads();
  if (i >= g.L) return;
  // (3) dV_j (lane = key j) = Σ_r P_rj dO_r over this wave's CV columns
  {
    float acc[CV];
#pragma unroll
    for (int c = 0; c < CV; ++c) acc[c] = 0.f;
#pragma unroll 8
    for (int r = 0; r < 64; ++r) {
      const float pr = pm[r][i];
#pragma unroll
      for (int c = 0; c < CV; c += 4) {
        const float4 d4 = *reinterpret_cast<const float4*>(&d[r][w * CV + c]);
        acc[c] = fmaf(pr, d4.x, acc[c]); acc[c + 1] = fmaf(pr, d4.y, acc[c + 1]);
        acc[c + 2] = fmaf(pr, d4.z, acc[c + 2]); acc[c + 3] = fmaf(pr, d4.w, acc[c + 3]);
      }
    }
    float* dst = g.dv + (seq * g.L + i) * g.ld_dv + head * DV + w * CV;
#pragma unroll
    for (int c = 0; c < CV; c += 4) *reinterpret_cast<float4*>(dst + c) = make_float4(acc[c], acc[c + 1], acc[c + 2], acc[c + 3]);
  }
  // (4) dKp_i = Σ_j (dS_ij + dS_ji) Kp_j over this wave's CK columns
  {
    float acc[CK];
#pragma unroll
    for (int c = 0; c < CK; ++c) acc[c] = 0.f;
#pragma unroll 8
    for (int j = 0; j < 64; ++j) {
      const float wgt = ds[i][j] + ds[j][i];
#pragma unroll
      for (int c = 0; c < CK; c += 4) {
        const float4 kj = *reinterpret_cast<const float4*>(&k[j][w * CK + c]);
        acc[c] = fmaf(wgt, kj.x, acc[c]); acc[c + 1] = fmaf(wgt, kj.y, acc[c + 1]);
        acc[c + 2] = fmaf(wgt, kj.z, acc[c + 2]); acc[c + 3] = fmaf(wgt, kj.w, acc[c + 3]);
      }
    }
    float* dst = g.out + (seq * g.L + i) * g.ld_out + head * DK + w * CK;
#pragma unroll
    for (int c = 0; c < CK; c += 4) *reinterpret_cast<float4*>(dst + c) = make_float4(acc[c], acc[c + 1], acc[c + 2], acc[c + 3]);
  }
}

template <int LMAX, int DK, int DV>
int launch(const AttnArgs& g, bool bwd, hipStream_t s) {
  constexpr int HPW = 64 / LMAX;
  if constexpr (LMAX == 64 && DK % (4 * SPLIT_NW) == 0 && DV % (4 * SPLIT_NW) == 0) {
    const dim3 grid((unsigned)g.nseq, (unsigned)g.heads);
    if (bwd)
      hipLaunchKernelGGL((mha_attn_bwd_split_kernel<DK, DV>), grid, dim3(64 * SPLIT_NW), 0, s, g);
    else
      hipLaunchKernelGGL((mha_attn_fwd_split_kernel<DK, DV>), grid, dim3(64 * SPLIT_NW), 0, s, g);
    NR_LAUNCH_CHECK();
    return NR_OK;
  }
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
