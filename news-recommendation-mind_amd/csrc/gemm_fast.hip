// Fast path of nr_gemm_f32: the same contraction as gemm_f32.hip with every operand mode a
// compile-time parameter, branch-free loads and per-tile row pointers hoisted out of the
// k-loop (gather / conv3 token rows are constant along k), so the loop body is loads, LDS
// stores and MFMAs only.
//
// LDS images, by operand layout:
//   K-contiguous operand (rows = M/N index, k contiguous in memory): [row][k], stride 36
//     floats — a 16-B ds_write per float4 and ONE ds_read_b128 per 4 MFMA k-steps; the
//     32-row lane groups of a b128 read hit 16 distinct 16-B slots (36/4 = 9 is odd).
//   MN-contiguous operand (rows = k): [k][row], stride R+4 — a 16-B store per float4 and
//     four ds_read_b32 per 4 k-steps (lanes read consecutive rows: conflict-free).
// MFMA k-step s (0..15) of a 32-deep tile reads k = 16*half + s in BOTH operands (the sum over
// k is order-free), which is what makes the b128 fragment read possible.
//
// Requirements (checked by the dispatcher, else the generic kernel runs): data 16-B aligned,
// ld % 4 == 0, MN-contiguous operands with ld >= round4(M or N) (reads stay inside padded
// rows), conv3 seg % 32 == 0 and seg % BN == 0 where the taps run along N.
#include "common.h"
#include "../../include/newsrec_hip.h"
#include "gemm_fast.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace nrfast {

// operand modes
enum { KC_PLAIN = 0, KC_GATHER = 1, KC_CONV3 = 2, MN_PLAIN = 3, MN_GATHER = 4, MN_CONV3 = 5 };

constexpr bool is_kc(int m) { return m <= KC_CONV3; }

struct Op {
  const float* base;
  int64_t ld;
  const int64_t* idx;
  int L;
  int seg;
};

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

// Register-staged tile loader for an operand of R rows (the M or N extent) x 32 k.
template <int R, int MODE>
struct Loader {
  static constexpr bool KC = is_kc(MODE);
  static constexpr int NV = R / 32;              // float4 per thread
  static constexpr int S = KC ? 36 : R + 4;      // LDS stride
  static constexpr int LDS_FLOATS = KC ? R * 36 : 32 * (R + 4);
  float4 v[NV];
  // K-contiguous: per-thread row bases (hoisted); conv3: the three tap token ids
  const float* rowp[NV];
  int64_t nbase[NV];     // conv3: first token row of the row's news
  int tpos[NV];          // conv3: position in the news
  uint32_t okbits;       // conv3: rows whose tap t+j-1 exists
  int curj;              // conv3: tap the row pointers are set up for
  int64_t kcol[NV];      // MN_GATHER: token ids of the next tile's rows (prefetched)

  __device__ __forceinline__ void init(const Op& d, int64_t r0, int64_t rlim, int tid) {
    if (KC) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int f = tid + 256 * i;
        int64_t row = r0 + (f >> 3);
        row = row < rlim ? row : rlim - 1;                  // clamp: rows >= M are discarded
        if (MODE == KC_PLAIN) rowp[i] = d.base + row * d.ld;
        if (MODE == KC_GATHER) rowp[i] = d.base + d.idx[row] * d.ld;
        if (MODE == KC_CONV3) {
          const int64_t n = row / d.L;
          nbase[i] = n * d.L;
          tpos[i] = (int)(row - n * d.L);
        }
      }
      curj = -1;
      okbits = 0;
    }
  }

  // conv3: point every row at tap j (token t+j-1 of its news; offset so that column k maps
  // to k - j*seg).  Runs when the k-tile crosses into a new tap: 3 times per block.
  __device__ __forceinline__ void set_tap(const Op& d, int j) {
    okbits = 0;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int t2 = tpos[i] + j - 1;
      const bool ok = t2 >= 0 && t2 < d.L;
      const int64_t tok = ok ? d.idx[nbase[i] + t2] : 0;
      rowp[i] = d.base + tok * d.ld - (int64_t)j * d.seg;
      okbits |= (ok ? 1u : 0u) << i;
    }
    curj = j;
  }

  // column offset (k) within the row for K-contiguous; r0 = tile's first row/col
  // Full 32-deep tiles only (the dispatcher requires K % 32 == 0): no per-element branches,
  // so hipcc keeps every load in flight across the MFMAs of the current tile.
  __device__ __forceinline__ void load(const Op& d, int64_t r0, int64_t rlim, int64_t k0, int tid) {
    if (MODE == KC_CONV3) {
      const int j = (int)(k0 / d.seg);
      if (j != curj) set_tap(d, j);
    }
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int f = tid + 256 * i;
      if (KC) {
        const int kq = f & 7;
        const int64_t k = k0 + 4 * kq;
        const float* p = rowp[i] + k;
        const bool ok = MODE != KC_CONV3 || ((okbits >> i) & 1u);
        float4 x = *reinterpret_cast<const float4*>(p);
        if (MODE == KC_CONV3 && !ok) x = make_float4(0.f, 0.f, 0.f, 0.f);
        v[i] = x;
      } else {
        constexpr int CPR = R / 4;
        const int kr = f / CPR, c4 = f % CPR;
        const int64_t k = k0 + kr;
        int64_t col = r0 + 4 * c4;
        const int64_t cmax = ((rlim + 3) & ~int64_t(3)) - 4;
        col = col < cmax ? col : cmax;                      // clamp inside the padded row
        const int64_t kk = k;
        const float* p;
        bool ok = true;
        if (MODE == MN_PLAIN) {
          p = d.base + kk * d.ld + col;
        } else if (MODE == MN_GATHER) {
          p = d.base + kcol[i] * d.ld + col;
        } else {   // MN_CONV3: rows = tokens, columns = tap*seg + e
          const int j = (int)(r0 / d.seg);
          const int64_t n = kk / d.L;
          const int t2 = (int)(kk - n * d.L) + j - 1;
          ok = t2 >= 0 && t2 < d.L;
          const int64_t tok = ok ? d.idx[n * d.L + t2] : 0;
          p = d.base + tok * d.ld + (col - (int64_t)j * d.seg);
        }
        float4 x = *reinterpret_cast<const float4*>(p);
        if (!ok) x = make_float4(0.f, 0.f, 0.f, 0.f);
        v[i] = x;
      }
    }
  }

  // MN_GATHER: fetch the token ids of tile k0's rows (one tile ahead of its data loads)
  __device__ __forceinline__ void prefetch_idx(const Op& d, int64_t k0, int64_t K, int tid) {
    if (MODE == MN_GATHER) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int f = tid + 256 * i;
        constexpr int CPR = R / 4;
        const int64_t k = k0 + f / CPR;
        kcol[i] = d.idx[k < K ? k : K - 1];
      }
    }
  }

  __device__ __forceinline__ void store(float* lds, int tid) const {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int f = tid + 256 * i;
      if (KC) {
        *reinterpret_cast<float4*>(&lds[(f >> 3) * 36 + 4 * (f & 7)]) = v[i];
      } else {
        constexpr int CPR = R / 4;
        *reinterpret_cast<float4*>(&lds[(f / CPR) * S + 4 * (f % CPR)]) = v[i];
      }
    }
  }

  // the 4 operand values of k-steps 4q..4q+3 for tile row `row` (lane half h)
  __device__ __forceinline__ float4 frag(const float* lds, int row, int h, int q) const {
    if (KC) return *reinterpret_cast<const float4*>(&lds[row * 36 + 16 * h + 4 * q]);
    const int k = 16 * h + 4 * q;
    return make_float4(lds[k * S + row], lds[(k + 1) * S + row], lds[(k + 2) * S + row], lds[(k + 3) * S + row]);
  }
};

template <int BM, int BN, int AM, int BMODE>
__global__ __launch_bounds__(256, 2) void gemm_fast_kernel(Args g) {
  using LA = Loader<BM, AM>;
  using LB = Loader<BN, BMODE>;
  __shared__ __attribute__((aligned(16))) float As[2][LA::LDS_FLOATS];
  __shared__ __attribute__((aligned(16))) float Bs[2][LB::LDS_FLOATS];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, c = lane & 31;
  const int64_t gm = (g.M + BM - 1) / BM, gn = (g.N + BN - 1) / BN;
  const int nwg = (int)(gm * gn);
  const int id = blockIdx.x;
  const int xcd = id & 7, q8 = nwg >> 3, rr = nwg & 7;
  const int wg = (xcd < rr ? xcd * (q8 + 1) : rr * (q8 + 1) + (xcd - rr) * q8) + (id >> 3);
  const int64_t m0 = (wg / gn) * BM, n0 = (wg % gn) * BN;
  const int64_t kbeg = (int64_t)blockIdx.y * g.kchunk;
  const int64_t kend = kbeg + g.kchunk < g.K ? kbeg + g.kchunk : g.K;
  const int nt = kend > kbeg ? (int)((kend - kbeg + 31) / 32) : 0;

  constexpr int TI = BM / 64, TJ = BN / 64;
  const int wm = (w >> 1) * (BM / 2), wn = (w & 1) * (BN / 2);
  f32x16 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  LA la;
  LB lb;
  la.init(g.A, m0, g.M, tid);
  lb.init(g.B, n0, g.N, tid);
  if (nt > 0) {
    la.prefetch_idx(g.A, kbeg, g.K, tid);
    lb.prefetch_idx(g.B, kbeg, g.K, tid);
    la.load(g.A, m0, g.M, kbeg, tid);
    lb.load(g.B, n0, g.N, kbeg, tid);
    if (nt > 1) {
      la.prefetch_idx(g.A, kbeg + 32, g.K, tid);
      lb.prefetch_idx(g.B, kbeg + 32, g.K, tid);
    }
    la.store(As[0], tid);
    lb.store(Bs[0], tid);
  }
  __syncthreads();

  for (int t = 0; t < nt; ++t) {
    const int buf = t & 1;
    if (t + 1 < nt) {
      const int64_t k1 = kbeg + (int64_t)(t + 1) * 32;
      la.load(g.A, m0, g.M, k1, tid);
      lb.load(g.B, n0, g.N, k1, tid);
      if (t + 2 < nt) {
        la.prefetch_idx(g.A, k1 + 32, g.K, tid);
        lb.prefetch_idx(g.B, k1 + 32, g.K, tid);
      }
    }
    const float* a_s = As[buf];
    const float* b_s = Bs[buf];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float4 a[TI], b[TJ];
#pragma unroll
      for (int i = 0; i < TI; ++i) a[i] = la.frag(a_s, wm + 32 * i + c, h, q);
#pragma unroll
      for (int j = 0; j < TJ; ++j) b[j] = lb.frag(b_s, wn + 32 * j + c, h, q);
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].x, b[j].x, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].y, b[j].y, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].z, b[j].z, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].w, b[j].w, acc[i][j], 0, 0, 0);
        }
    }
    if (t + 1 < nt) {
      la.store(As[buf ^ 1], tid);
      lb.store(Bs[buf ^ 1], tid);
    }
    __syncthreads();
  }

#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int64_t col = n0 + wn + 32 * j + c;
      if (col >= g.N) continue;
      const bool has_bias = g.bias && (g.epi == NR_EPI_STORE || g.epi == NR_EPI_STORE_RELU ||
                                       g.epi == NR_EPI_STORE_TANH || g.epi == NR_EPI_ACCUM);
      const float bcol = has_bias ? g.bias[col] : 0.f;
      int sj = 0;
      int64_t scol = col;
      if (g.epi == NR_EPI_SCATTER && g.Cm.L > 0 && g.Cm.seg > 0 && g.Cm.idx && g.Cm.L != 1) {
        sj = (int)(col / g.Cm.seg);
        scol = col - (int64_t)sj * g.Cm.seg;
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (row >= g.M) continue;
        const float v = acc[i][j][r];
        const int64_t o = row * g.ldc + col;
        switch (g.epi) {
          case NR_EPI_STORE: g.C[o] = v + bcol; break;
          case NR_EPI_STORE_RELU: g.C[o] = fmaxf(v + bcol, 0.f); break;
          case NR_EPI_STORE_TANH: g.C[o] = tanhf(v + bcol); break;
          case NR_EPI_ACCUM: g.C[o] += v + bcol; break;
          case NR_EPI_ACCUM_GATE: g.C[o] = g.Cm.base[row * g.Cm.ld + col] > 0.f ? g.C[o] + v : 0.f; break;
          case NR_EPI_ATOMIC: atomicAdd(&g.C[o], v); break;
          default: {   // NR_EPI_SCATTER through a GATHER (L == 1) or CONV3 row map
            int64_t tok;
            if (g.Cm.L == 1) {
              tok = g.Cm.idx[row];
            } else {
              const int64_t n = row / g.Cm.L;
              const int t2 = (int)(row - n * g.Cm.L) + sj - 1;
              if (t2 < 0 || t2 >= g.Cm.L) continue;
              tok = g.Cm.idx[n * g.Cm.L + t2];
            }
            if (tok == g.pad_row) continue;
            atomicAdd(&g.C[tok * g.ldc + scol], v);
          }
        }
      }
    }
}

template <int BM, int BN, int AM, int BMODE>
int launch(const Args& g, int splits, hipStream_t s) {
  const int64_t gm = (g.M + BM - 1) / BM, gn = (g.N + BN - 1) / BN;
  hipLaunchKernelGGL((gemm_fast_kernel<BM, BN, AM, BMODE>), dim3((unsigned)(gm * gn), (unsigned)splits), dim3(256),
                     0, s, g);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

template <int BM, int BN>
int launch_modes(const Args& g, int am, int bm, int splits, hipStream_t s) {
#define NR_AB(A_, B_) \
  if (am == A_ && bm == B_) return launch<BM, BN, A_, B_>(g, splits, s);
  NR_AB(KC_GATHER, KC_PLAIN)   // fused gather + projection (fwd)
  NR_AB(KC_CONV3, KC_PLAIN)    // conv as K = 3E GEMM (fwd)
  NR_AB(KC_PLAIN, KC_PLAIN)    // plain y = x Wᵀ
  NR_AB(KC_PLAIN, MN_PLAIN)    // dgrad dx = dy W
  NR_AB(MN_PLAIN, MN_GATHER)   // wgrad dW = dyᵀ table[ids]
  NR_AB(MN_PLAIN, MN_CONV3)    // conv wgrad
  NR_AB(MN_PLAIN, MN_PLAIN)    // wgrad dW = dyᵀ x
#undef NR_AB
  return -1;
}

}  // namespace nrfast

// Returns -1 if the shape/operands are not eligible (the caller falls back), else a status.
int nr_gemm_fast(int64_t M, int64_t N, int64_t K, const nr_operand* A, const nr_operand* B, float* C,
                 int64_t ldc, const float* bias, int32_t epilogue, const nr_operand* c_rows, int64_t pad_row,
                 int32_t split_k, int bm, int bn, hipStream_t stream) {
  using namespace nrfast;
  auto aligned = [](const nr_operand* o) {
    return (o->ld % 4 == 0) && ((reinterpret_cast<uintptr_t>(o->data) & 15) == 0);
  };
  if (!aligned(A) || !aligned(B) || (K % 32)) return -1;
  int am, bmode;
  if (A->layout == NR_KCONTIG) {
    am = A->map == NR_ROWS_PLAIN ? KC_PLAIN : A->map == NR_ROWS_GATHER ? KC_GATHER : KC_CONV3;
    if (am == KC_CONV3 && (A->seg % 32)) return -1;
  } else {
    if (A->map != NR_ROWS_PLAIN || A->ld < ((M + 3) & ~3LL)) return -1;
    am = MN_PLAIN;
  }
  if (B->layout == NR_KCONTIG) {
    if (B->map != NR_ROWS_PLAIN) return -1;
    bmode = KC_PLAIN;
  } else {
    bmode = B->map == NR_ROWS_PLAIN ? MN_PLAIN : B->map == NR_ROWS_GATHER ? MN_GATHER : MN_CONV3;
    if (B->ld < ((N + 3) & ~3LL) && bmode != MN_CONV3) return -1;
    if (bmode == MN_CONV3 && (B->seg % bn || B->seg % 4)) return -1;
  }
  Args g;
  g.M = M; g.N = N; g.K = K;
  g.A = Op{A->data, A->ld, A->rows, A->seq_len, A->seg};
  g.B = Op{B->data, B->ld, B->rows, B->seq_len, B->seg};
  g.Cm = Op{c_rows ? c_rows->data : nullptr, c_rows ? c_rows->ld : 0, c_rows ? c_rows->rows : nullptr,
            c_rows ? (c_rows->map == NR_ROWS_CONV3 ? c_rows->seq_len : 1) : 1, c_rows ? c_rows->seg : 1};
  if (epilogue == NR_EPI_SCATTER && c_rows && c_rows->map == NR_ROWS_PLAIN) return -1;
  if (epilogue == NR_EPI_SCATTER && c_rows && c_rows->map == NR_ROWS_CONV3 && c_rows->seq_len == 1) return -1;
  g.C = C; g.ldc = ldc; g.bias = bias; g.epi = epilogue; g.pad_row = pad_row;
  g.kchunk = (K + split_k - 1) / split_k;
  g.kchunk = (g.kchunk + 31) / 32 * 32;
  if (g.kchunk == 0) g.kchunk = 32;
  const int splits = (int)((K + g.kchunk - 1) / g.kchunk) > 0 ? (int)((K + g.kchunk - 1) / g.kchunk) : 1;
  if (bm == 128 && bn == 128) return launch_modes<128, 128>(g, am, bmode, splits, stream);
  if (bm == 64 && bn == 64) return launch_modes<64, 64>(g, am, bmode, splits, stream);
  return -1;
}
