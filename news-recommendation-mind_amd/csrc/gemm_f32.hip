// fp32 GEMM on the CDNA4 f32-input matrix cores (v_mfma_f32_32x32x2_f32: exact f32,
// 64 FLOP/clk/SIMD, the same rate as the f32 VALU but with one VGPR per operand per lane).
//
// It carries every dense contraction of the news / user towers:
//   * the MHA key/value projections   (models/Modules/Attention.py:107-108, :125-127)
//   * the k=3 Conv1d of the CNN encoder as a GEMM with K = 3E  (models/Encoders/CNN.py:12-17,41)
//   * their backward dgrad / wgrad     (autograd of the above)
// The word-embedding gather (models/Embeddings/BERT.py:39) is FUSED into the operand loader:
// an operand row can be a token id's row of the [V, E] table (GATHER), or the three
// neighbouring tokens of a k=3 convolution with zero padding at the title ends (CONV3), so the
// [T, 768] embedding activations are never written to HBM.  The dgrad epilogue scatters
// straight back into the dense [V, E] table gradient with no-return f32 atomics, skipping the
// padding row (nn.Embedding padding_idx=0).
//
// Tile: BM x BN x 32, 256 threads = 4 waves in 2x2, each wave (BM/2) x (BN/2) of 32x32 MFMA
// tiles.  Operands are register-staged into a double-buffered LDS image laid out [k][m]
// (m contiguous) so each lane's fragment is one ds_read_b32 per k-pair; the next tile's global
// loads are issued before the current tile's MFMAs.  Blocks are remapped XCD-aware so that the
// column tiles of one row panel run on the same XCD and share its L2.
#include "common.h"
#include "../../include/newsrec_hip.h"
#include "gemm_fast.h"
#include <stdlib.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

struct Op {
  const float* base;
  int64_t ld;
  const int64_t* idx;
  int map;
  int L;
  int seg;
  int vec;   // rows 16-B aligned: float4 loads; else scalar loads
};

__device__ __forceinline__ const float* row_ptr(const Op& d, int64_t r, int j) {
  if (d.map == NR_ROWS_PLAIN) return d.base + r * d.ld;
  if (d.map == NR_ROWS_GATHER) return d.base + d.idx[r] * d.ld;
  // CONV3: row r = (news n, position t); tap j reads position t + j - 1 (zero outside)
  int64_t n = r / d.L;
  int t2 = (int)(r - n * d.L) + j - 1;
  if (t2 < 0 || t2 >= d.L) return nullptr;
  return d.base + d.idx[n * d.L + t2] * d.ld;
}

struct Args {
  int64_t M, N, K;
  Op A, B, Cm;
  float* C;
  int64_t ldc;
  const float* bias;
  int epi;
  int64_t pad_row;
  int64_t kchunk;
};

// Loads one operand tile (R rows of the M/N side x 32 k) into registers.
// KC = true : element (r, k) stored at row_ptr(r)[k]  (k contiguous)
// KC = false: element (r, k) stored at row_ptr(k)[r]  (r contiguous)
template <int R, bool KC>
struct Tile {
  static constexpr int BK = 32;
  static constexpr int NV = R / 32;                 // float4 per thread
  static constexpr int S = KC ? R + 1 : R + 4;      // LDS row stride ([k][r] image)
  float4 v[NV];

  __device__ __forceinline__ void load(const Op& d, int64_t r0, int64_t rlim, int64_t k0,
                                       int64_t K, int tid) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int f = tid + 256 * i;
      float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
      if (KC) {
        const int r = f >> 3, kq = f & 7;
        const int64_t row = r0 + r, k = k0 + 4 * kq;
        const int j = d.map == NR_ROWS_CONV3 ? (int)(k0 / d.seg) : 0;
        if (row < rlim && k < K) {
          const float* p = row_ptr(d, row, j);
          if (p) {
            p += k - (int64_t)j * d.seg;
            if (k + 3 < K && d.vec) {
              x = *reinterpret_cast<const float4*>(p);
            } else if (k + 3 < K) {
              x.x = p[0]; x.y = p[1]; x.z = p[2]; x.w = p[3];
            } else {
              x.x = p[0];
              if (k + 1 < K) x.y = p[1];
              if (k + 2 < K) x.z = p[2];
            }
          }
        }
      } else {
        constexpr int CPR = R / 4;                    // float4 per k-row
        const int kr = f / CPR, c4 = f % CPR;
        const int64_t k = k0 + kr, col = r0 + 4 * c4;
        const int j = d.map == NR_ROWS_CONV3 ? (int)(r0 / d.seg) : 0;
        if (k < K && col < rlim) {
          const float* p = row_ptr(d, k, j);
          if (p) {
            p += col - (int64_t)j * d.seg;
            if (col + 3 < rlim && d.vec) {
              x = *reinterpret_cast<const float4*>(p);
            } else if (col + 3 < rlim) {
              x.x = p[0]; x.y = p[1]; x.z = p[2]; x.w = p[3];
            } else {
              x.x = p[0];
              if (col + 1 < rlim) x.y = p[1];
              if (col + 2 < rlim) x.z = p[2];
            }
          }
        }
      }
      v[i] = x;
    }
  }

  __device__ __forceinline__ void store(float* lds, int tid) const {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int f = tid + 256 * i;
      if (KC) {
        const int r = f >> 3, kq = f & 7;
        lds[(4 * kq + 0) * S + r] = v[i].x;
        lds[(4 * kq + 1) * S + r] = v[i].y;
        lds[(4 * kq + 2) * S + r] = v[i].z;
        lds[(4 * kq + 3) * S + r] = v[i].w;
      } else {
        constexpr int CPR = R / 4;
        const int kr = f / CPR, c4 = f % CPR;
        *reinterpret_cast<float4*>(&lds[kr * S + 4 * c4]) = v[i];
      }
    }
  }
};

template <int BM, int BN, bool AK, bool BKC>
__global__ __launch_bounds__(256, 2) void gemm_f32_kernel(Args g) {
  constexpr int BK = 32;
  using TA = Tile<BM, AK>;
  using TB = Tile<BN, BKC>;
  __shared__ __attribute__((aligned(16))) float As[2][BK * TA::S];
  __shared__ __attribute__((aligned(16))) float Bs[2][BK * TB::S];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t gm = (g.M + BM - 1) / BM, gn = (g.N + BN - 1) / BN;
  const int nwg = (int)(gm * gn);
  const int id = blockIdx.x;
  // bijective XCD remap: blocks id, id+8, ... share an XCD; give them consecutive tiles
  const int xcd = id & 7, q = nwg >> 3, rr = nwg & 7;
  const int wg = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (id >> 3);
  const int64_t m0 = (wg / gn) * BM, n0 = (wg % gn) * BN;

  const int64_t kbeg = (int64_t)blockIdx.y * g.kchunk;
  const int64_t kend = kbeg + g.kchunk < g.K ? kbeg + g.kchunk : g.K;
  const int nt = kend > kbeg ? (int)((kend - kbeg + BK - 1) / BK) : 0;

  constexpr int TI = BM / 64, TJ = BN / 64;
  const int wm = (w >> 1) * (BM / 2), wn = (w & 1) * (BN / 2);
  f32x16 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  TA ta;
  TB tb;
  if (nt > 0) {
    ta.load(g.A, m0, g.M, kbeg, g.K, tid);
    tb.load(g.B, n0, g.N, kbeg, g.K, tid);
    ta.store(As[0], tid);
    tb.store(Bs[0], tid);
  }
  __syncthreads();

  for (int t = 0; t < nt; ++t) {
    const int buf = t & 1;
    if (t + 1 < nt) {
      ta.load(g.A, m0, g.M, kbeg + (int64_t)(t + 1) * BK, g.K, tid);
      tb.load(g.B, n0, g.N, kbeg + (int64_t)(t + 1) * BK, g.K, tid);
    }
    const float* a_s = As[buf];
    const float* b_s = Bs[buf];
#pragma unroll
    for (int kk = 0; kk < BK / 2; ++kk) {
      const int kr = 2 * kk + (lane >> 5);
      float a[TI], b[TJ];
#pragma unroll
      for (int i = 0; i < TI; ++i) a[i] = a_s[kr * TA::S + wm + 32 * i + (lane & 31)];
#pragma unroll
      for (int j = 0; j < TJ; ++j) b[j] = b_s[kr * TB::S + wn + 32 * j + (lane & 31)];
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (t + 1 < nt) {
      ta.store(As[buf ^ 1], tid);
      tb.store(Bs[buf ^ 1], tid);
    }
    __syncthreads();
  }

  // epilogue: 32x32 C/D map — col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int64_t col = n0 + wn + 32 * j + (lane & 31);
      if (col >= g.N) continue;
      const float bcol = (g.bias && (g.epi == NR_EPI_STORE || g.epi == NR_EPI_STORE_RELU ||
                                     g.epi == NR_EPI_STORE_TANH || g.epi == NR_EPI_ACCUM ||
                                     g.epi == NR_EPI_STORE_GELU)) ? g.bias[col] : 0.f;
      int sj = 0;
      int64_t scol = col;
      if (g.epi == NR_EPI_SCATTER && g.Cm.map == NR_ROWS_CONV3) {
        sj = (int)(col / g.Cm.seg);
        scol = col - (int64_t)sj * g.Cm.seg;
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (row >= g.M) continue;
        const float v = acc[i][j][r];
        if (g.epi == NR_EPI_STORE) {
          g.C[row * g.ldc + col] = v + bcol;
        } else if (g.epi == NR_EPI_STORE_RELU) {
          g.C[row * g.ldc + col] = fmaxf(v + bcol, 0.f);
        } else if (g.epi == NR_EPI_STORE_TANH) {
          g.C[row * g.ldc + col] = tanhf(v + bcol);
        } else if (g.epi == NR_EPI_ACCUM_GATE) {
          const int64_t o = row * g.ldc + col;
          g.C[o] = g.Cm.base[row * g.Cm.ld + col] > 0.f ? g.C[o] + v : 0.f;
        } else if (g.epi == NR_EPI_ACCUM) {
          g.C[row * g.ldc + col] += v + bcol;
        } else if (g.epi == NR_EPI_STORE_GELU) {
          const float x = v + bcol;
          const_cast<float*>(g.Cm.base)[row * g.Cm.ld + col] = x;
          g.C[row * g.ldc + col] = nr_gelu(x);
        } else if (g.epi == NR_EPI_GELU_GRAD) {
          g.C[row * g.ldc + col] = v * nr_gelu_grad(g.Cm.base[row * g.Cm.ld + col]);
        } else if (g.epi == NR_EPI_ATOMIC) {
          atomicAdd(&g.C[row * g.ldc + col], v);
        } else {  // NR_EPI_SCATTER
          int64_t tok;
          if (g.Cm.map == NR_ROWS_GATHER) {
            tok = g.Cm.idx[row];
          } else if (g.Cm.map == NR_ROWS_CONV3) {
            const int64_t n = row / g.Cm.L;
            const int t2 = (int)(row - n * g.Cm.L) + sj - 1;
            if (t2 < 0 || t2 >= g.Cm.L) continue;
            tok = g.Cm.idx[n * g.Cm.L + t2];
          } else {
            tok = row;
          }
          if (tok == g.pad_row) continue;
          atomicAdd(&g.C[tok * g.ldc + scol], v);
        }
      }
    }
}

Op to_op(const nr_operand* o) {
  Op d;
  d.base = o ? o->data : nullptr;
  d.ld = o ? o->ld : 0;
  d.idx = o ? o->rows : nullptr;
  d.map = o ? o->map : NR_ROWS_PLAIN;
  d.L = o ? o->seq_len : 1;
  d.seg = o ? o->seg : 1;
  d.vec = o && (o->ld % 4 == 0) && ((reinterpret_cast<uintptr_t>(o->data) & 15) == 0);
  return d;
}

template <int BM, int BN, bool AK, bool BKC>
int launch(const Args& g, int splits, hipStream_t s) {
  const int64_t gm = (g.M + BM - 1) / BM, gn = (g.N + BN - 1) / BN;
  dim3 grid((unsigned)(gm * gn), (unsigned)splits);
  hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, AK, BKC>), grid, dim3(256), 0, s, g);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

template <int BM, int BN>
int launch_kc(const Args& g, int ak, int bk, int splits, hipStream_t s) {
  if (ak && bk) return launch<BM, BN, true, true>(g, splits, s);
  if (ak && !bk) return launch<BM, BN, true, false>(g, splits, s);
  if (!ak && bk) return launch<BM, BN, false, true>(g, splits, s);
  return launch<BM, BN, false, false>(g, splits, s);
}

int pick_tile(int64_t n) {  // 64 or 128: least padding, ties -> 128
  const int64_t p64 = (n + 63) / 64 * 64, p128 = (n + 127) / 128 * 128;
  return p128 <= p64 ? 128 : 64;
}

}  // namespace

namespace {
int gemm_static(int64_t M, int64_t N, int64_t K, const nr_operand* A, const nr_operand* B, float* C, int64_t ldc,
                const float* bias, int32_t epilogue, const nr_operand* c_rows, int64_t pad_row, int32_t split_k,
                int32_t prec, float* work, int64_t work_elems, float* colsum, int32_t* colsum_folded,
                hipStream_t stream) {
  if (M < 0 || N < 0 || K < 0) return NR_EINVAL(0);
  if (prec != NR_GEMM_F32 && prec != NR_GEMM_BF16X6 && prec != NR_GEMM_BF16) return NR_EINVAL(12);
  if (epilogue < NR_EPI_STORE || epilogue > NR_EPI_SCATTER_ZEROED) return NR_EINVAL(3);
  if (!A || !B || !C || !A->data || !B->data) return NR_EINVAL(1);
  if (((A->map != NR_ROWS_PLAIN) && (A->ld & 3)) || ((B->map != NR_ROWS_PLAIN) && (B->ld & 3)))
    return NR_EINVAL(2);   // gathered tables must be float4-addressable
  if (epilogue == NR_EPI_SCATTER && (!c_rows || (c_rows->map != NR_ROWS_PLAIN && !c_rows->rows)))
    return NR_EINVAL(4);
  if ((epilogue == NR_EPI_ACCUM_GATE || epilogue == NR_EPI_STORE_GELU || epilogue == NR_EPI_GELU_GRAD) &&
      (!c_rows || !c_rows->data))
    return NR_EINVAL(4);
  if (split_k < 1) split_k = 1;
  if (split_k > 1 && epilogue != NR_EPI_ATOMIC && epilogue != NR_EPI_SCATTER) return NR_EINVAL(5);
  if (M == 0 || N == 0) return NR_OK;

  Args g;
  g.M = M; g.N = N; g.K = K;
  g.A = to_op(A); g.B = to_op(B); g.Cm = to_op(c_rows);
  g.C = C; g.ldc = ldc; g.bias = bias; g.epi = epilogue; g.pad_row = pad_row;
  g.kchunk = (K + split_k - 1) / split_k;
  g.kchunk = (g.kchunk + 31) / 32 * 32;
  if (g.kchunk == 0) g.kchunk = 32;
  const int splits = (int)((K + g.kchunk - 1) / g.kchunk) > 0 ? (int)((K + g.kchunk - 1) / g.kchunk) : 1;

  if ((epilogue == NR_EPI_SCATTER_STORE || epilogue == NR_EPI_SCATTER_ZEROED) &&
      (!c_rows || c_rows->map != NR_ROWS_GATHER || !c_rows->rows))
    return NR_EINVAL(4);
  {
    const int64_t t128 = ((M + 127) / 128) * ((N + 127) / 128) * splits;
    // bf16x6 and f32: small problems (< 400 tiles of 128x128) take 64x64 tiles, which only the
    // exact-f32 kernel has (they are latency-bound, and 128x128 tiles would leave most CUs idle);
    // larger ones take 128x128 tiles (bf16x6: the split kernels; f32: the exact-f32 128x128 kernel).
    // bf16: every eligible shape runs on the bf16 kernel (one product per tile is cheap).
    const int64_t small_min = 400;
    const int fb = (prec == NR_GEMM_BF16 || t128 >= small_min) ? 128 : 64;
    const int rc = nr_gemm_fast(M, N, K, A, B, C, ldc, bias, epilogue, c_rows, pad_row, split_k, fb, fb, nullptr,
                                nullptr, prec, 0, work, work_elems, colsum, colsum_folded, stream);
    if (rc != -1) return rc;
  }
  // generic kernel: same sums via atomics
  if (epilogue == NR_EPI_SCATTER_STORE || epilogue == NR_EPI_SCATTER_ZEROED) g.epi = NR_EPI_SCATTER;
  int bm = pick_tile(M), bn = pick_tile(N);
  // small problems: prefer 64x64 tiles to fill the 256 CUs
  if ((int64_t)((M + bm - 1) / bm) * ((N + bn - 1) / bn) * splits < 512) { bm = 64; bn = 64; }
  // CONV3 operands need a tap-uniform tile: seg must be a multiple of the tile extent
  // along the axis that carries the taps (k for K-contiguous, m/n otherwise)
  const int ak = A->layout == NR_KCONTIG;
  const int bk = B->layout == NR_KCONTIG;
  if (A->map == NR_ROWS_CONV3 && ak && (A->seg % 32)) return NR_EINVAL(6);
  if (B->map == NR_ROWS_CONV3 && bk && (B->seg % 32)) return NR_EINVAL(6);
  if (A->map == NR_ROWS_CONV3 && !ak && (A->seg % bm)) bm = 64;
  if (B->map == NR_ROWS_CONV3 && !bk && (B->seg % bn)) bn = 64;
  if ((A->map == NR_ROWS_CONV3 && !ak && (A->seg % bm)) ||
      (B->map == NR_ROWS_CONV3 && !bk && (B->seg % bn)))
    return NR_EINVAL(7);
  if (bm == 128 && bn == 128) return launch_kc<128, 128>(g, ak, bk, splits, stream);
  if (bm == 128 && bn == 64) return launch_kc<128, 64>(g, ak, bk, splits, stream);
  if (bm == 64 && bn == 128) return launch_kc<64, 128>(g, ak, bk, splits, stream);
  return launch_kc<64, 64>(g, ak, bk, splits, stream);
}

int gemm_dyn(int64_t M, int64_t N, int64_t K, const nr_operand* A, const nr_operand* B, float* C, int64_t ldc,
             const float* bias, int32_t epilogue, const nr_operand* c_rows, int64_t pad_row, int32_t split_k,
             const int32_t* m_dev, const int32_t* k_dev, int32_t prec, int32_t max_cus, float* work,
             int64_t work_elems, float* colsum, int32_t* colsum_folded, hipStream_t stream);
}  // namespace

extern "C" int nr_gemm_f32(int64_t M, int64_t N, int64_t K, const nr_operand* A,
                           const nr_operand* B, float* C, int64_t ldc, const float* bias,
                           int32_t epilogue, const nr_operand* c_rows, int64_t pad_row,
                           int32_t split_k, int32_t prec, hipStream_t stream) {
  return gemm_static(M, N, K, A, B, C, ldc, bias, epilogue, c_rows, pad_row, split_k, prec, nullptr, 0, nullptr,
                     nullptr, stream);
}

extern "C" int nr_gemm_f32_ws(int64_t M, int64_t N, int64_t K, const nr_operand* A, const nr_operand* B, float* C,
                              int64_t ldc, const float* bias, int32_t epilogue, const nr_operand* c_rows,
                              int64_t pad_row, int32_t split_k, const int32_t* m_dev, const int32_t* k_dev,
                              int32_t prec, int32_t max_cus, float* work, int64_t work_elems, float* colsum,
                              int32_t* colsum_folded, hipStream_t stream) {
  if (work_elems < 0 || (work_elems > 0 && !work)) return NR_EINVAL(16);
  if (colsum_folded) *colsum_folded = 0;
  if (colsum && !colsum_folded) return NR_EINVAL(17);
  if (!m_dev && !k_dev && max_cus == 0)
    return gemm_static(M, N, K, A, B, C, ldc, bias, epilogue, c_rows, pad_row, split_k, prec, work, work_elems,
                       colsum, colsum_folded, stream);
  return gemm_dyn(M, N, K, A, B, C, ldc, bias, epilogue, c_rows, pad_row, split_k, m_dev, k_dev, prec, max_cus, work,
                  work_elems, colsum, colsum_folded, stream);
}

// Device-resident extents: M and K are upper bounds (grid sizing); the kernel reads the actual
// values from m_dev / k_dev (either may be null).  Fast-path operand shapes only (K-contiguous
// or MN-contiguous rows, 16-B aligned, ld % 4 == 0); the device K must be a multiple of 32.
extern "C" int nr_gemm_f32_dyn(int64_t M, int64_t N, int64_t K, const nr_operand* A, const nr_operand* B,
                               float* C, int64_t ldc, const float* bias, int32_t epilogue,
                               const nr_operand* c_rows, int64_t pad_row, int32_t split_k, const int32_t* m_dev,
                               const int32_t* k_dev, int32_t prec, hipStream_t stream) {
  return nr_gemm_f32_dyn_cus(M, N, K, A, B, C, ldc, bias, epilogue, c_rows, pad_row, split_k, m_dev, k_dev, prec, 0,
                             stream);
}

extern "C" int nr_gemm_f32_dyn_cus(int64_t M, int64_t N, int64_t K, const nr_operand* A, const nr_operand* B,
                                   float* C, int64_t ldc, const float* bias, int32_t epilogue,
                                   const nr_operand* c_rows, int64_t pad_row, int32_t split_k, const int32_t* m_dev,
                                   const int32_t* k_dev, int32_t prec, int32_t max_cus, hipStream_t stream) {
  return gemm_dyn(M, N, K, A, B, C, ldc, bias, epilogue, c_rows, pad_row, split_k, m_dev, k_dev, prec, max_cus,
                  nullptr, 0, nullptr, nullptr, stream);
}

namespace {
int gemm_dyn(int64_t M, int64_t N, int64_t K, const nr_operand* A, const nr_operand* B, float* C, int64_t ldc,
             const float* bias, int32_t epilogue, const nr_operand* c_rows, int64_t pad_row, int32_t split_k,
             const int32_t* m_dev, const int32_t* k_dev, int32_t prec, int32_t max_cus, float* work,
             int64_t work_elems, float* colsum, int32_t* colsum_folded, hipStream_t stream) {
  if (max_cus < 0) return NR_EINVAL(15);
  if (M < 0 || N < 0 || K < 0 || (K % 32)) return NR_EINVAL(0);
  if (prec != NR_GEMM_F32 && prec != NR_GEMM_BF16X6 && prec != NR_GEMM_BF16) return NR_EINVAL(14);
  if (epilogue < NR_EPI_STORE || epilogue > NR_EPI_SCATTER_ZEROED) return NR_EINVAL(3);
  if (!A || !B || !C || !A->data || !B->data) return NR_EINVAL(1);
  if ((A->ld & 3) || (B->ld & 3)) return NR_EINVAL(2);
  if (epilogue == NR_EPI_SCATTER && (!c_rows || (c_rows->map != NR_ROWS_PLAIN && !c_rows->rows)))
    return NR_EINVAL(4);
  if ((epilogue == NR_EPI_ACCUM_GATE || epilogue == NR_EPI_STORE_GELU || epilogue == NR_EPI_GELU_GRAD) &&
      (!c_rows || !c_rows->data))
    return NR_EINVAL(4);
  if ((epilogue == NR_EPI_SCATTER_STORE || epilogue == NR_EPI_SCATTER_ZEROED) &&
      (!c_rows || c_rows->map != NR_ROWS_GATHER || !c_rows->rows))
    return NR_EINVAL(4);
  if (split_k < 1) split_k = 1;
  if (split_k > 1 && epilogue != NR_EPI_ATOMIC && epilogue != NR_EPI_SCATTER) return NR_EINVAL(5);
  if (M == 0 || N == 0 || K == 0) return NR_OK;
  const int rc = nr_gemm_fast(M, N, K, A, B, C, ldc, bias, epilogue, c_rows, pad_row, split_k, 128, 128, m_dev,
                              k_dev, prec, max_cus, work, work_elems, colsum, colsum_folded, stream);
  return rc == -1 ? NR_EINVAL(7) : rc;
}
}  // namespace
