// Shared device code of the fast GEMM kernels (gemm_fast.hip: exact f32 MFMA; gemm_split.hip:
// bf16x6): operand loaders, LDS images, epilogues, the persistent tile scheduler.  Internal.
#pragma once
#include <stdlib.h>

#include "common.h"
#include "../../include/newsrec_hip.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

namespace nrfast {

// ---- bf16x6 arithmetic: fp32 operands as three bf16 terms (x = h + m + l to 2^-24 |x|) and six
// products a_h b_h + a_h b_m + a_m b_h + a_h b_l + a_m b_m + a_l b_h on v_mfma_f32_32x32x16_bf16
// (16x the f32 MFMA rate); the dropped terms are O(2^-24) of |a b|, like the f32 MFMA rounding.
__device__ __forceinline__ uint32_t bf_rne(float x) {
  const uint32_t u = __float_as_uint(x);
  return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
}
__device__ __forceinline__ float bf_f(uint32_t b) { return __uint_as_float(b << 16); }
// hardware conversions, two values per v_cvt_pk_bf16_f32 (round to nearest even); a packed pair's
// bf16 halves widen back to fp32 with one shift / mask each
__device__ __forceinline__ uint32_t bf_bits(__bf16 v) { return (uint32_t)__builtin_bit_cast(uint16_t, v); }
typedef float nr_f2 __attribute__((ext_vector_type(2)));
typedef __bf16 nr_b2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((nr_f2){a, b}, nr_b2));
}
__device__ __forceinline__ float pk_lo(uint32_t p) { return __uint_as_float(p << 16); }
__device__ __forceinline__ float pk_hi(uint32_t p) { return __uint_as_float(p & 0xffff0000u); }
// a, b -> the packed (h, m, l) terms of both: 3 conversions, 4 bit ops, 4 subtractions per pair
// (the bf16x6 GEMM units build without SLP vectorisation so these subtractions stay scalar
// v_sub_f32 beside the MFMAs: build.py EXTRA)
__device__ __forceinline__ void split2(float a, float b, uint32_t& h, uint32_t& m, uint32_t& l) {
  h = pk_bf16(a, b);
  const float ra = a - pk_lo(h), rb = b - pk_hi(h);   // exact
  m = pk_bf16(ra, rb);
  l = pk_bf16(ra - pk_lo(m), rb - pk_hi(m));
}
__device__ __forceinline__ void split4(float a, float b, float c, float d, uint2& p0, uint2& p1, uint2& p2) {
  split2(a, b, p0.x, p1.x, p2.x);
  split2(c, d, p0.y, p1.y, p2.y);
}
// bf16 arithmetic (one product): the four values rounded to bf16 (RNE), packed
__device__ __forceinline__ uint2 hi4(float a, float b, float c, float d) {
  return make_uint2(pk_bf16(a, b), pk_bf16(c, d));
}
constexpr int SROW = 40;          // split LDS image: [plane][row][k] bf16, 32 k + 8 pad (80-B rows)
constexpr int SPL = 128 * SROW;   // one plane of a 128-row operand tile

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
  int vec;   // float4 epilogue: N, ldc (and aux ld) % 4 == 0, C (and aux) 16-B aligned
  int splits;
  const int32_t* mdyn;   // device-resident M (<= M), or null
  const int32_t* kdyn;   // device-resident K (<= K), or null
  int tail;  // big kernel, NR_EPI_SCATTER_ZEROED: max K pieces of the last partial round's tiles (0 = off)
  // big kernel, the stream-K tail through the workspace (slab with tail): partial tiles the workspace
  // holds; the plan keeps rem * pieces <= tail_cap whatever the grid (occupancy > 1 per CU included)
  int tail_cap = 0;
  int max_cus;   // persistent grid limited to this many CUs (0 = all): leaves CUs to a concurrent collective
  // big kernel, split-K NR_EPI_ATOMIC: each split stores its partial tile to slab + split * slab_stride
  // ([M][slab_ld], plain stores) and splitk_reduce adds the splits into C -- instead of fp32 atomics
  float* slab = nullptr;
  int64_t slab_ld = 0, slab_stride = 0;
  // slab path with an MN-contiguous A (a weight gradient dYᵀ X): the units of the first column tile
  // also sum A over their k range (the bias gradient, from the tiles they load anyway) into
  // slab[splits * slab_stride + split * (slab_stride / slab_ld) + m]; splitk_reduce adds them to colsum
  float* colsum = nullptr;
};

// CUs of the current device (cached)
inline int device_cus() {
  static int cache[16] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return 0;
  if (cache[dev] == 0) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    cache[dev] = cus;
  }
  return cache[dev];
}

// persistent grid of `slots` resident workgroups (all CUs) capped to max_cus CUs' worth
inline int capped_slots(int slots, int max_cus) {
  const int cus = device_cus();
  if (max_cus <= 0 || cus <= 0 || max_cus >= cus || slots <= 0) return slots;
  const int per = slots / cus > 0 ? slots / cus : 1;
  return per * max_cus;
}

// K-contiguous 32-deep tile: float4 f (of R x 8) holds k quad kc_quad(f) of row kc_row(f).  Each
// 64-float4 block covers 8 rows; the lanes of one 16-lane ds_write_b64 group take rows g and g + 4
// (SROW = 20 dwords: 0 and 16 mod 32), so the split-stores hit 32 distinct banks (consecutive rows
// 0 and 1 would share banks 0-3; MI355X_MICROARCH.md §LDS).  Each 8-lane group is one whole row, so
// the fp32 image's ds_write_b128 stays conflict-free too.
__device__ __forceinline__ int kc_row(int f) { return 8 * (f >> 6) + ((f & 63) >> 4) + 4 * ((f >> 3) & 1); }
__device__ __forceinline__ int kc_quad(int f) { return f & 7; }

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
        int64_t row = r0 + kc_row(f);
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
        const int kq = kc_quad(f);
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
        *reinterpret_cast<float4*>(&lds[kc_row(f) * 36 + 4 * kc_quad(f)]) = v[i];
      } else {
        constexpr int CPR = R / 4;
        *reinterpret_cast<float4*>(&lds[(f / CPR) * S + 4 * (f % CPR)]) = v[i];
      }
    }
  }

  // split LDS image (K-contiguous operands only): the float4 of 4 k of one row -> NP planes
  // (NP = 3: bf16x6 terms h, m, l; NP = 1: bf16 arithmetic, the value rounded to bf16)
  template <int NP>
  __device__ __forceinline__ void store_split(uint16_t* lds, int tid) const {
    if constexpr (KC) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int f = tid + 256 * i;
        uint16_t* q = lds + kc_row(f) * SROW + 4 * kc_quad(f);
        if constexpr (NP == 1) {
          *reinterpret_cast<uint2*>(q) = hi4(v[i].x, v[i].y, v[i].z, v[i].w);
        } else {
          uint2 p0, p1, p2;
          split4(v[i].x, v[i].y, v[i].z, v[i].w, p0, p1, p2);
          *reinterpret_cast<uint2*>(q) = p0;
          *reinterpret_cast<uint2*>(q + SPL) = p1;
          *reinterpret_cast<uint2*>(q + 2 * SPL) = p2;
        }
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

// bf16x6 loader of an MN-contiguous 128-row operand (stored rows = k): thread (kg = tid & 7,
// cg = tid >> 3) loads the 4x4 block k0+4kg.., columns r0+4cg.. as 4 float4 (8 lanes cover 128
// contiguous bytes of a stored row), transposes it in registers and writes each column's 4
// consecutive k to the [row][k] planes (b64 stores, 2-way bank aliasing).
template <int MODE>
struct MNBlk {
  static_assert(MODE == MN_PLAIN || MODE == MN_GATHER || MODE == MN_CONV3, "MNBlk: plain, gathered or conv3 rows");
  float4 v[4];
  int64_t kid[4];   // MN_GATHER: stored-row ids of the next tile (prefetched)

  __device__ __forceinline__ void init(const Op&, int64_t, int64_t, int) {}

  __device__ __forceinline__ void load(const Op& d, int64_t r0, int64_t rlim, int64_t k0, int tid) {
    const int kg = tid & 7, cg = tid >> 3;
    int64_t col = r0 + 4 * cg;
    const int64_t cmax = ((rlim + 3) & ~int64_t(3)) - 4;
    col = col < cmax ? col : cmax;   // clamp inside the padded row; rows >= M are discarded
    if (MODE == MN_CONV3) {   // stored rows = tokens, columns = tap * seg + e (the tile is within one tap)
      const int j = (int)(r0 / d.seg);
      const int64_t ecol = col - (int64_t)j * d.seg;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t kk = k0 + 4 * kg + u;
        const int64_t n = kk / d.L;
        const int t2 = (int)(kk - n * d.L) + j - 1;
        const bool ok = t2 >= 0 && t2 < d.L;
        const int64_t tok = ok ? d.idx[n * d.L + t2] : 0;
        v[u] = *reinterpret_cast<const float4*>(d.base + tok * d.ld + ecol);
        if (!ok) v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
      return;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t row = MODE == MN_PLAIN ? k0 + 4 * kg + u : kid[u];
      v[u] = *reinterpret_cast<const float4*>(d.base + row * d.ld + col);
    }
  }

  __device__ __forceinline__ void prefetch_idx(const Op& d, int64_t k0, int64_t K, int tid) {
    if (MODE == MN_GATHER) {
      const int kg = tid & 7;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t k = k0 + 4 * kg + u;
        kid[u] = d.idx[k < K ? k : K - 1];
      }
    }
  }

  template <int NP>
  __device__ __forceinline__ void put(uint16_t* q, float a, float b, float c, float e) const {
    if constexpr (NP == 1) {
      *reinterpret_cast<uint2*>(q) = hi4(a, b, c, e);
    } else {
      uint2 p0, p1, p2;
      split4(a, b, c, e, p0, p1, p2);
      *reinterpret_cast<uint2*>(q) = p0;
      *reinterpret_cast<uint2*>(q + SPL) = p1;
      *reinterpret_cast<uint2*>(q + 2 * SPL) = p2;
    }
  }

  template <int NP>
  __device__ __forceinline__ void store_split(uint16_t* lds, int tid) const {
    const int kg = tid & 7, cg = tid >> 3;
    uint16_t* q = lds + (4 * cg) * SROW + 4 * kg;
    put<NP>(q, v[0].x, v[1].x, v[2].x, v[3].x);
    put<NP>(q + SROW, v[0].y, v[1].y, v[2].y, v[3].y);
    put<NP>(q + 2 * SROW, v[0].z, v[1].z, v[2].z, v[3].z);
    put<NP>(q + 3 * SROW, v[0].w, v[1].w, v[2].w, v[3].w);
  }
};

// Output-tile epilogue.  The MFMAs run with the operands swapped (B tile as the "A" operand),
// so each accumulator holds a Cᵀ tile: lane (c, h) owns output row m = c of the 32x32 tile
// and, in register group q = r >> 2, the four consecutive columns n = 8q + 4h .. +3 — one
// float4 per group.  Per wave: TI*TJ*4 vector stores (vs 64 scalar stores in the C-major
// layout), one bias float4 per group, one token-id lookup per row for the scatter.
template <int EPI>
__device__ __forceinline__ float4 epi_combine(const Args& g, float4 v, float4 b, const float* crow, const float* arow,
                                              int64_t n) {
  if (EPI == NR_EPI_STORE) return make_float4(v.x + b.x, v.y + b.y, v.z + b.z, v.w + b.w);
  if (EPI == NR_EPI_STORE_RELU)
    return make_float4(fmaxf(v.x + b.x, 0.f), fmaxf(v.y + b.y, 0.f), fmaxf(v.z + b.z, 0.f), fmaxf(v.w + b.w, 0.f));
  if (EPI == NR_EPI_STORE_TANH) return make_float4(tanhf(v.x + b.x), tanhf(v.y + b.y), tanhf(v.z + b.z), tanhf(v.w + b.w));
  if (EPI == NR_EPI_ACCUM) {
    const float4 o = *reinterpret_cast<const float4*>(crow + n);
    return make_float4(o.x + v.x + b.x, o.y + v.y + b.y, o.z + v.z + b.z, o.w + v.w + b.w);
  }
  if (EPI == NR_EPI_GELU_GRAD) {
    const float4 a = *reinterpret_cast<const float4*>(arow + n);
    return make_float4(v.x * nr_gelu_grad(a.x), v.y * nr_gelu_grad(a.y), v.z * nr_gelu_grad(a.z),
                       v.w * nr_gelu_grad(a.w));
  }
  // NR_EPI_ACCUM_GATE
  const float4 o = *reinterpret_cast<const float4*>(crow + n);
  const float4 a = *reinterpret_cast<const float4*>(arow + n);
  return make_float4(a.x > 0.f ? o.x + v.x : 0.f, a.y > 0.f ? o.y + v.y : 0.f, a.z > 0.f ? o.z + v.z : 0.f,
                     a.w > 0.f ? o.w + v.w : 0.f);
}

template <int EPI>
__device__ __forceinline__ float epi_combine1(const Args& g, float v, float b, const float* crow, const float* arow,
                                              int64_t n) {
  if (EPI == NR_EPI_STORE) return v + b;
  if (EPI == NR_EPI_STORE_RELU) return fmaxf(v + b, 0.f);
  if (EPI == NR_EPI_STORE_TANH) return tanhf(v + b);
  if (EPI == NR_EPI_ACCUM) return crow[n] + v + b;
  if (EPI == NR_EPI_GELU_GRAD) return v * nr_gelu_grad(arow[n]);
  return arow[n] > 0.f ? crow[n] + v : 0.f;
}

template <int EPI, int TI, int TJ>
__device__ __forceinline__ void epilogue_t(const Args& g, f32x16 (&acc)[TI][TJ], int64_t m0, int64_t n0, int wm,
                                           int wn, int h, int c, bool vec) {
  const bool has_bias = g.bias && (EPI == NR_EPI_STORE || EPI == NR_EPI_STORE_RELU || EPI == NR_EPI_STORE_TANH ||
                                   EPI == NR_EPI_ACCUM || EPI == NR_EPI_STORE_GELU);
#pragma unroll
  for (int i = 0; i < TI; ++i) {
    const int64_t row = m0 + wm + 32 * i + c;
    if (row >= g.M) continue;
    float* crow = g.C + row * g.ldc;
    if (EPI == NR_EPI_SCATTER_STORE) {   // distinct destination rows: plain stores
      const int64_t tok = g.Cm.idx[row];
      if (tok == g.pad_row) continue;
      crow = g.C + tok * g.ldc;
    }
    const float* arow =
        (EPI == NR_EPI_ACCUM_GATE || EPI == NR_EPI_GELU_GRAD || EPI == NR_EPI_STORE_GELU) ? g.Cm.base + row * g.Cm.ld
                                                                                          : nullptr;
    int64_t tok = 0, nbase = 0;
    int tpos = 0;
    if (EPI == NR_EPI_SCATTER) {
      if (g.Cm.L == 1) {
        tok = g.Cm.idx[row];
      } else {
        nbase = row / g.Cm.L;
        tpos = (int)(row - nbase * g.Cm.L);
        nbase *= g.Cm.L;
      }
    }
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t n = n0 + wn + 32 * j + 8 * q + 4 * h;
        if (n >= g.N) continue;
        const float4 v = make_float4(acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]);
        if (EPI == NR_EPI_ATOMIC || EPI == NR_EPI_SCATTER) {
          float* dst;
          int64_t t = tok;
          int64_t sn = n;
          if (EPI == NR_EPI_ATOMIC) {
            dst = crow;
          } else {
            if (g.Cm.L != 1) {   // conv3 row map: column tap sj of token t + sj - 1
              const int sj = (int)(n / g.Cm.seg);
              sn = n - (int64_t)sj * g.Cm.seg;
              const int t2 = tpos + sj - 1;
              if (t2 < 0 || t2 >= g.Cm.L) continue;
              t = g.Cm.idx[nbase + t2];
            }
            if (t == g.pad_row) continue;
            dst = g.C + t * g.ldc;
          }
          const float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (n + u < g.N) atomicAdd(dst + sn + u, e[u]);
        } else if (EPI == NR_EPI_SCATTER_STORE) {
          if (vec && n + 3 < g.N) {
            *reinterpret_cast<float4*>(crow + n) = v;
          } else {
            const float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int u = 0; u < 4; ++u)
              if (n + u < g.N) crow[n + u] = e[u];
          }
        } else if (EPI == NR_EPI_STORE_GELU) {   // pre-activation to aux, GELU to C
          float* xrow = const_cast<float*>(arow);
          const float e[4] = {v.x, v.y, v.z, v.w};
          if (vec && n + 3 < g.N) {
            const float4 b = has_bias ? *reinterpret_cast<const float4*>(g.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
            const float4 x = make_float4(v.x + b.x, v.y + b.y, v.z + b.z, v.w + b.w);
            *reinterpret_cast<float4*>(xrow + n) = x;
            *reinterpret_cast<float4*>(crow + n) = make_float4(nr_gelu(x.x), nr_gelu(x.y), nr_gelu(x.z), nr_gelu(x.w));
          } else {
#pragma unroll
            for (int u = 0; u < 4; ++u)
              if (n + u < g.N) {
                const float x = e[u] + (has_bias ? g.bias[n + u] : 0.f);
                xrow[n + u] = x;
                crow[n + u] = nr_gelu(x);
              }
          }
        } else if (vec && n + 3 < g.N) {
          const float4 b = has_bias ? *reinterpret_cast<const float4*>(g.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
          *reinterpret_cast<float4*>(crow + n) = epi_combine<EPI>(g, v, b, crow, arow, n);
        } else {
          const float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (n + u < g.N) crow[n + u] = epi_combine1<EPI>(g, e[u], has_bias ? g.bias[n + u] : 0.f, crow, arow, n + u);
        }
      }
  }
}

// Atomic epilogues in the C-major accumulator layout (operands not swapped): lane c owns
// column n = c, register r row (r & 3) + 8 (r >> 2) + 4h — each atomic instruction covers 32
// consecutive columns of two rows (two cache lines), 16x fewer line transactions than the
// transposed layout would issue.
template <int EPI, int TI, int TJ>
__device__ __forceinline__ void epilogue_cmajor(const Args& g, f32x16 (&acc)[TI][TJ], int64_t m0, int64_t n0, int wm,
                                                int wn, int h, int c) {
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int64_t col = n0 + wn + 32 * j + c;
      if (col >= g.N) continue;
      int sj = 0;
      int64_t scol = col;
      if (EPI == NR_EPI_SCATTER && g.Cm.L != 1) {
        sj = (int)(col / g.Cm.seg);
        scol = col - (int64_t)sj * g.Cm.seg;
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (row >= g.M) continue;
        const float v = acc[i][j][r];
        if (EPI == NR_EPI_ATOMIC) {
          atomicAdd(&g.C[row * g.ldc + col], v);
        } else {
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

// Split-K partial tile -> its slab with plain stores, in the C-major accumulator layout (each store
// instruction writes 32 consecutive columns of two rows).
template <int TI, int TJ>
__device__ __forceinline__ void epilogue_slab(const Args& g, f32x16 (&acc)[TI][TJ], int64_t m0, int64_t n0, int wm,
                                              int wn, int h, int c, float* dst) {
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int64_t col = n0 + wn + 32 * j + c;
      if (col >= g.N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (row < g.M) dst[row * g.slab_ld + col] = acc[i][j][r];
      }
    }
}

template <int TI, int TJ>
__device__ __forceinline__ void epilogue(const Args& g, f32x16 (&acc)[TI][TJ], int64_t m0, int64_t n0, int wm,
                                         int wn, int h, int c) {
  const bool vec = g.vec;
  switch (g.epi) {
    case NR_EPI_STORE: epilogue_t<NR_EPI_STORE, TI, TJ>(g, acc, m0, n0, wm, wn, h, c, vec); break;
    case NR_EPI_STORE_RELU: epilogue_t<NR_EPI_STORE_RELU, TI, TJ>(g, acc, m0, n0, wm, wn, h, c, vec); break;
    case NR_EPI_STORE_TANH: epilogue_t<NR_EPI_STORE_TANH, TI, TJ>(g, acc, m0, n0, wm, wn, h, c, vec); break;
    case NR_EPI_ACCUM: epilogue_t<NR_EPI_ACCUM, TI, TJ>(g, acc, m0, n0, wm, wn, h, c, vec); break;
    case NR_EPI_ACCUM_GATE: epilogue_t<NR_EPI_ACCUM_GATE, TI, TJ>(g, acc, m0, n0, wm, wn, h, c, vec); break;
    case NR_EPI_STORE_GELU: epilogue_t<NR_EPI_STORE_GELU, TI, TJ>(g, acc, m0, n0, wm, wn, h, c, vec); break;
    case NR_EPI_GELU_GRAD: epilogue_t<NR_EPI_GELU_GRAD, TI, TJ>(g, acc, m0, n0, wm, wn, h, c, vec); break;
    case NR_EPI_ATOMIC: epilogue_t<NR_EPI_ATOMIC, TI, TJ>(g, acc, m0, n0, wm, wn, h, c, vec); break;
    case NR_EPI_SCATTER_STORE: epilogue_t<NR_EPI_SCATTER_STORE, TI, TJ>(g, acc, m0, n0, wm, wn, h, c, vec); break;
    default: epilogue_t<NR_EPI_SCATTER, TI, TJ>(g, acc, m0, n0, wm, wn, h, c, vec); break;
  }
}

template <bool TR, int TI, int TJ>
__device__ __forceinline__ void epilogue_any(const Args& g, f32x16 (&acc)[TI][TJ], int64_t m0, int64_t n0, int wm,
                                             int wn, int h, int c) {
  if (TR) {
    epilogue<TI, TJ>(g, acc, m0, n0, wm, wn, h, c);
  } else if (g.epi == NR_EPI_ATOMIC) {
    epilogue_cmajor<NR_EPI_ATOMIC, TI, TJ>(g, acc, m0, n0, wm, wn, h, c);
  } else {
    epilogue_cmajor<NR_EPI_SCATTER, TI, TJ>(g, acc, m0, n0, wm, wn, h, c);
  }
}

// Floats before the big kernel's tail partial tiles in its NR_EPI_SCATTER_ZEROED workspace (ints
// {full, rem, pieces, gn} of the launch's stream-K tail, padded to 256 B; gemm_big_impl.h tail_slab_tr)
constexpr int TAIL_WS_HDR = 64;

// A work unit = one BM x BN output tile x one K split.
struct Unit {
  int64_t m0, n0, kbeg;
  int nt;   // 32-deep k-tiles
};

// Virtual block id -> unit.  Ids congruent mod 8 run on the same XCD (the hardware deals
// workgroups round-robin over the 8 XCDs); each XCD gets a contiguous run of units, n fastest,
// so the blocks resident on one XCD at a time share A row panels (and all of B) in its L2.
__device__ __forceinline__ Unit decode_unit(const Args& g, int id, int units, int ntiles, int gn, int BM, int BN) {
  const int xcd = id & 7, q8 = units >> 3, rr = units & 7;
  const int u = (xcd < rr ? xcd * (q8 + 1) : rr * (q8 + 1) + (xcd - rr) * q8) + (id >> 3);
  const int tile = u % ntiles, split = u / ntiles;
  Unit r;
  r.m0 = (int64_t)(tile / gn) * BM;
  r.n0 = (int64_t)(tile % gn) * BN;
  r.kbeg = (int64_t)split * g.kchunk;
  const int64_t kend = r.kbeg + g.kchunk < g.K ? r.kbeg + g.kchunk : g.K;
  r.nt = kend > r.kbeg ? (int)((kend - r.kbeg + 31) / 32) : 0;
  return r;
}

// Position in a block's flattened (unit, k-tile) sequence.
struct Cursor {
  int id;   // virtual block id (units of this block: blockIdx.x + j * gridDim.x)
  int kt;   // k-tile within the unit
  Unit u;
};

// Resident-block slots for a kernel instantiation (CUs x occupancy), cached per device.
template <typename Kern>
int resident_slots(Kern k) {
  static int cache[16] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return 0;
  if (cache[dev] == 0) {
    int cus = 0, per = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k, 256, 0) != hipSuccess) return 0;
    cache[dev] = cus * per;
  }
  return cache[dev];
}

// bf16 launches of the 128x128 fast-path operand combinations (gemm_split_*.hip), np = 3 (bf16x6)
// or 1 (bf16); -1 = not covered
int launch_split_modes(const Args& g, int am, int bm, int splits, int np, hipStream_t s);

}  // namespace nrfast
