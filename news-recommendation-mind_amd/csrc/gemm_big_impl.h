// Large-tile bf16 matrix-core GEMM (bf16x6: NP = 3 planes, six products; bf16: NP = 1), included by
// the gemm_big_*.hip translation units.  Same operand modes, epilogues, persistent XCD-aware unit
// order and C ABI semantics as the 128x128 kernel (gemm_split_impl.h); built for the big
// contractions of the step (the news-tower projection and its dgrad / wgrad, the BERT dense layers).
//
// Why a second kernel: at 128x128 every fp32 element loaded feeds 2x fewer MFMAs, and the per-tile
// split (fp32 -> three bf16 terms) costs ~10 VALU per MFMA; with two workgroups per CU phase-locked
// on two barriers per k-step the VALU and the matrix cores barely overlap (MFMA busy 0.37,
// profiles/pmc_proj_fwd.json).  Here:
//   * 256 x BN tile (BN = 256 or 128), 8 waves (512 threads), wave tile 128x64 or 64x64: each loaded
//     element feeds twice the MFMAs, halving the split work per MFMA;
//   * 16-deep k-tiles, LDS DOUBLE-buffered ([stage][plane][row][24] bf16, 48-B rows: ds_read_b128
//     fragments conflict-free; the K-contiguous split-stores conflict-free by their row order,
//     BigKC), ONE barrier per k-tile: while the waves run k-tile P's MFMAs from
//     one stage, the same waves split k-tile P+1 (already in registers) into the other stage and
//     issue the global loads of P+2, so the VALU / LDS-store / load work is interleaved with the
//     MFMA stream of the same wave instead of being serialised between barriers;
//   * one workgroup per CU (147 KiB of LDS at BN = 256), persistent over the (tile, k-split) units.
#pragma once
#include <type_traits>

#include "gemm_fast_common.h"

namespace nrfast {

constexpr int BIG_BM = 256;
// k-tile depth: bf16x6 (three planes) 16; bf16 (one plane) 32 when both operands are K-contiguous --
// twice the MFMAs between barriers in the same LDS budget -- else 16: the MN-contiguous loaders'
// stores at 32 cost more than the extra MFMAs per barrier buy (one-box A/B, bf16, µs: BERT FFN-in
// weight gradient 657 -> 387, NRMS table dgrad 208 -> 141, CNN conv weight gradient 144 -> 115;
// the K-contiguous forward shapes keep 32: BERT FFN-out 152 vs 187 at 16)
template <int NP, int AM, int BMODE>
constexpr int big_bk() { return NP == 1 && is_kc(AM) && is_kc(BMODE) ? 32 : 16; }
// bf16 per LDS row: BK k + 8 pad (48 / 80 B: odd multiples of 16 B, conflict-free ds_read_b128)
template <int BK>
constexpr int big_sr() { return BK + 8; }

// K-contiguous operand, R rows x BK k: 512 threads x (R BK / 2048) float4.  Float4 f holds k quad
// quad_of(f) of tile row row_of(f); each 64-float4 block covers 64 / QPR consecutive rows.  The
// split-stores are ds_write_b64 (one 4-k bf16 quad per plane), serviced in four 16-lane groups over
// 32 banks (MI355X_MICROARCH.md §LDS): a group must cover 32 distinct banks.  With rows of SR bf16
// (12 dwords at BK = 16, 20 at BK = 32) a group of consecutive rows wraps onto itself (rows 0 and 3
// share banks 4-7 at BK = 16; rows 0 and 1 banks 0-3 at BK = 32: the 2-way conflicts the round-3
// PMC counted, ~2 extra cycles per LDS instruction), so a group takes rows 12 dwords x {0, 2, 4, 6}
// = {0, 24, 16, 8} mod 32 apart (BK = 16: rows of one parity) or 20 x {0, 4} = {0, 16} (BK = 32).
template <int R, int MODE, int BK>
struct BigKC {
  static constexpr int QPR = BK / 4;           // float4 per row
  static constexpr int NV = R * QPR / 512;
  static constexpr int SR = big_sr<BK>();
  static_assert(QPR == 4 || QPR == 8, "BigKC: 16- or 32-deep k-tiles");
  float4 v[2][NV];   // two register sets: k-tile t lives in set t % 2 (loads issued 3 tiles ahead)
  const float* rowp[NV];
  __device__ __forceinline__ static int row_of(int f) {
    const int l = f & 63, g = l >> 4;
    return QPR == 4 ? 16 * (f >> 6) + 8 * (g >> 1) + (g & 1) + 2 * ((l >> 2) & 3)
                    : 8 * (f >> 6) + g + 4 * ((l >> 3) & 1);
  }
  __device__ __forceinline__ static int quad_of(int f) { return f & (QPR - 1); }
  __device__ __forceinline__ void init(const Op& d, int64_t r0, int64_t rlim, int tid) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int f = tid + 512 * i;
      int64_t row = r0 + row_of(f);
      row = row < rlim ? row : rlim - 1;   // clamp: rows >= M are computed and discarded
      rowp[i] = MODE == KC_GATHER ? d.base + d.idx[row] * d.ld : d.base + row * d.ld;
    }
  }
  template <int S>
  __device__ __forceinline__ void prefetch_idx(const Op&, int64_t, int64_t, int) {}
  template <int S>
  __device__ __forceinline__ void load(const Op& d, int64_t, int64_t, int64_t k0, int tid) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int f = tid + 512 * i;
      v[S][i] = *reinterpret_cast<const float4*>(rowp[i] + k0 + 4 * quad_of(f));
    }
  }
  // float4 i of register set S -> its plane slots
  template <int S, int NP>
  __device__ __forceinline__ void store_one(uint16_t* lds, int tid, int i) const {
    constexpr int PL = R * SR;   // one plane
    const int f = tid + 512 * i;
    uint16_t* q = lds + row_of(f) * SR + 4 * quad_of(f);
    const float4 x = v[S][i];
    if constexpr (NP == 1) {
      *reinterpret_cast<uint2*>(q) = hi4(x.x, x.y, x.z, x.w);
    } else {
      uint2 p0, p1, p2;
      split4(x.x, x.y, x.z, x.w, p0, p1, p2);
      *reinterpret_cast<uint2*>(q) = p0;
      *reinterpret_cast<uint2*>(q + PL) = p1;
      *reinterpret_cast<uint2*>(q + 2 * PL) = p2;
    }
  }
  template <int S, int NP>
  __device__ __forceinline__ void store(uint16_t* lds, int tid) const {
#pragma unroll
    for (int i = 0; i < NV; ++i) store_one<S, NP>(lds, tid, i);
  }
  // piece p of PIECES equal parts of store() (the interleaved k-tile spreads them between MFMAs)
  static constexpr int PIECES = NV;
  template <int S, int NP>
  __device__ __forceinline__ void store_piece(uint16_t* lds, int tid, int p) const {
    store_one<S, NP>(lds, tid, p);
  }
};

// MN-contiguous operand (stored rows = k), R rows x BK k, in chunks of 2 (k) x 4 (row): chunk
// (kp, cg) = k0 + 2 kp + {0, 1}, rows r0 + 4 cg .. + 3, loaded as two float4; each row's two
// consecutive k go to LDS as one 32-bit word per plane.  Thread t takes chunks c = t + 2R j
// (kp = c & (BK/2 - 1) ... for BK = 16 the original mapping: kp = t & 7, cg = t >> 3).
template <int R, int MODE, int BK>
struct BigMN {
  static_assert(MODE == MN_PLAIN || MODE == MN_GATHER, "BigMN: plain or gathered stored rows");
  static constexpr int KP = BK / 2;                            // k pairs per tile
  static constexpr int CH = (R / 4) * KP;                      // chunks per tile
  static constexpr int NC = CH >= 512 ? CH / 512 : 1;          // chunks per thread
  // active threads.  The guards below test ACT < 512 first: with every thread active a runtime
  // `tid >= 512` (never true under __launch_bounds__(512), but not provable) put an exec-mask branch
  // around each load / split-store and broke the k-tile into blocks, with a vmcnt(0) at the top of
  // every tile -- the weight-gradient GEMMs ran 20 % slower than round 3 (profiles/r04_f_gemm_ab.json)
  static constexpr int ACT = CH >= 512 ? 512 : CH;
  static constexpr int SR = big_sr<BK>();
  static_assert(CH % 512 == 0 || CH < 512, "BigMN: whole chunks per thread");
  float4 v[2][NC][2];     // [register set][chunk][k of the pair]
  int64_t kid[2][NC][2];  // MN_GATHER: stored-row ids of a set's next tile (prefetched one load ahead)
  __device__ __forceinline__ void init(const Op&, int64_t, int64_t, int) {}
  // column sums of register set S's tile (both k of each pair), times f (0 or 1), into cs (the fused
  // bias gradient)
  template <int S>
  __device__ __forceinline__ void add_colsum(float (&cs)[NC][4], int tid, float f = 1.f) const {
    if (ACT < 512 && tid >= ACT) return;
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      // a select, not a multiply by f: a weighted-out tile (f = 0) holding an Inf must not add NaN
      cs[j][0] += f != 0.f ? v[S][j][0].x + v[S][j][1].x : 0.f;
      cs[j][1] += f != 0.f ? v[S][j][0].y + v[S][j][1].y : 0.f;
      cs[j][2] += f != 0.f ? v[S][j][0].z + v[S][j][1].z : 0.f;
      cs[j][3] += f != 0.f ? v[S][j][0].w + v[S][j][1].w : 0.f;
    }
  }
  // the per-thread sums of the KP threads of one column group (adjacent lanes) combined; the
  // group's first lane stores its four columns' sums (columns past M skipped)
  __device__ __forceinline__ void put_colsum(float (&cs)[NC][4], int64_t r0, int64_t rlim, float* dst,
                                             int tid) const {
    if (ACT < 512 && tid >= ACT) return;
#pragma unroll
    for (int j = 0; j < NC; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float x = cs[j][e];
#pragma unroll
        for (int d = 1; d < KP; d <<= 1) x += __shfl_xor(x, d, 64);
        cs[j][e] = x;
      }
    if (tid % KP) return;
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      const int64_t col = r0 + 4 * cg_of(tid + 512 * j);
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (col + e < rlim) dst[col + e] = cs[j][e];
    }
  }
  __device__ __forceinline__ static int kp_of(int c) { return c % KP; }
  __device__ __forceinline__ static int cg_of(int c) { return c / KP; }
  template <int S>
  __device__ __forceinline__ void prefetch_idx(const Op& d, int64_t k0, int64_t K, int tid) {
    if (MODE == MN_GATHER && (ACT == 512 || tid < ACT)) {
#pragma unroll
      for (int j = 0; j < NC; ++j)
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int64_t k = k0 + 2 * kp_of(tid + 512 * j) + u;
          kid[S][j][u] = d.idx[k < K ? k : K - 1];
        }
    }
  }
  template <int S>
  __device__ __forceinline__ void load(const Op& d, int64_t r0, int64_t rlim, int64_t k0, int tid) {
    if (ACT < 512 && tid >= ACT) return;
    const int64_t cmax = ((rlim + 3) & ~int64_t(3)) - 4;
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      const int c = tid + 512 * j;
      int64_t col = r0 + 4 * cg_of(c);
      col = col < cmax ? col : cmax;   // clamp inside the padded row; rows >= M are discarded
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int64_t row = MODE == MN_PLAIN ? k0 + 2 * kp_of(c) + u : kid[S][j][u];
        v[S][j][u] = *reinterpret_cast<const float4*>(d.base + row * d.ld + col);
      }
    }
  }
  template <int NP>
  __device__ __forceinline__ void put(uint16_t* q, float a, float b) const {
    constexpr int PL = R * SR;
    if constexpr (NP == 1) {
      *reinterpret_cast<uint32_t*>(q) = pk_bf16(a, b);
    } else {
      uint32_t hh, mm, ll;
      split2(a, b, hh, mm, ll);
      *reinterpret_cast<uint32_t*>(q) = hh;
      *reinterpret_cast<uint32_t*>(q + PL) = mm;
      *reinterpret_cast<uint32_t*>(q + 2 * PL) = ll;
    }
  }
  // Chunk (column group cg, k pair kp) writes its four rows 4cg .. 4cg + 3 as four ds_write_b32 per
  // plane.  At BK = 16 the row stride is 12 words, so row 4cg + i sits at bank 16 cg + 12 i + kp
  // (mod 32): in natural order the four column groups of a 32-lane half land on two bank windows (a
  // 2-way conflict on every write).  Column groups with cg ^ (cg >> 1) odd write their rows in the
  // order 2, 3, 0, 1 instead, which puts the four windows 8 banks apart: conflict-free.  (The float4
  // halves are swapped to match: 4 selects per float4.)
  // chunk j's rows 2 half .. 2 half + 1 (half 0: rows 0, 1 or 2, 3 per the rotation below)
  template <int S, int NP>
  __device__ __forceinline__ void store_half(uint16_t* lds, int tid, int j, int half) const {
    if (ACT < 512 && tid >= ACT) return;
    const int c = tid + 512 * j;
    const int cg = cg_of(c);
    const bool rot = BK == 16 && ((cg ^ (cg >> 1)) & 1) != 0;
    uint16_t* q = lds + (4 * cg) * SR + 2 * kp_of(c);
    const float4 a = v[S][j][0], b = v[S][j][1];
    if (half == 0) {
      uint16_t* qa = q + (rot ? 2 * SR : 0);   // rows 0, 1 (or 2, 3)
      put<NP>(qa, rot ? a.z : a.x, rot ? b.z : b.x);
      put<NP>(qa + SR, rot ? a.w : a.y, rot ? b.w : b.y);
    } else {
      uint16_t* qb = q + (rot ? 0 : 2 * SR);   // rows 2, 3 (or 0, 1)
      put<NP>(qb, rot ? a.x : a.z, rot ? b.x : b.z);
      put<NP>(qb + SR, rot ? a.y : a.w, rot ? b.y : b.w);
    }
  }
  // Chunk (column group cg, k pair kp) writes its four rows 4cg .. 4cg + 3 as four ds_write_b32 per
  // plane (see store_half for the order).
  template <int S, int NP>
  __device__ __forceinline__ void store(uint16_t* lds, int tid) const {
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      store_half<S, NP>(lds, tid, j, 0);
      store_half<S, NP>(lds, tid, j, 1);
    }
  }
  static constexpr int PIECES = 2 * NC;
  template <int S, int NP>
  __device__ __forceinline__ void store_piece(uint16_t* lds, int tid, int p) const {
    store_half<S, NP>(lds, tid, p >> 1, p & 1);
  }
};

template <int R, int MODE, int BK>
using BigLoader = typename std::conditional<is_kc(MODE), BigKC<R, MODE, BK>, BigMN<R, MODE, BK>>::type;

// Tail pieces through a workspace (NR_EPI_SCATTER_ZEROED with Args::slab): header ints {full, rem,
// pieces, gn} at slab[0..4) (block 0 writes them every launch), then one 256 x 256 partial tile per
// tail unit j = id - full at slab + TAIL_WS_HDR + j * 65536, row-major in the tile's local (row,
// column) -- stored with plain float4 stores in the transposed accumulator layout (lane (h, c) holds
// row c, columns 8q + 4h .. + 3).  tail_reduce_kernel adds a tile's pieces in piece order and stores
// the sums to their destination rows: deterministic, and no fp32 atomics (a round of 234 partial
// tiles added atomically cost ~47 us at the chip's ~1.3 TB/s atomic rate).
template <int TI, int TJ>
__device__ __forceinline__ void tail_slab_tr(f32x16 (&acc)[TI][TJ], int wm, int wn, int h, int c, float* dst) {
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        *reinterpret_cast<float4*>(dst + (wm + 32 * i + c) * 256 + wn + 32 * j + 8 * q + 4 * h) =
            make_float4(acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]);
}

// Atomic scatter-add of a tail piece in the transposed accumulator layout (lane (h, c) holds row c,
// columns 8q + 4h + 0..3 of each 32 x 32 block): one block at a time goes through LDS (waves 0-3 in
// the A image, 4-7 in the B image, 32 x 36 floats each) and is read back two rows x 32 consecutive
// columns per instruction, so each atomic instruction touches two cache lines instead of 32 (device
// atomics are resolved past the XCD's L2: their cost is per line, not per element).
template <int TI, int TJ>
__device__ __forceinline__ void tail_scatter_tr(const Args& g, f32x16 (&acc)[TI][TJ], int64_t m0, int64_t n0, int wm,
                                                int wn, int h, int c, int w, int lane, float* chunk) {
  constexpr int CS = 36;
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      __syncthreads();   // previous block read back (or the k-loop's last stage reads done)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        *reinterpret_cast<float4*>(chunk + c * CS + 8 * q + 4 * h) =
            make_float4(acc[i][j][4 * q], acc[i][j][4 * q + 1], acc[i][j][4 * q + 2], acc[i][j][4 * q + 3]);
      __syncthreads();
      const int64_t col = n0 + wn + 32 * j + (lane & 31);
#pragma unroll 4
      for (int rr = 0; rr < 16; ++rr) {
        const int rl = 2 * rr + (lane >> 5);
        const int64_t row = m0 + wm + 32 * i + rl;
        if (row >= g.M || col >= g.N) continue;
        const int64_t tok = g.Cm.idx[row];
        if (tok == g.pad_row) continue;
        atomicAdd(g.C + tok * g.ldc + col, chunk[rl * CS + (lane & 31)]);
      }
    }
  (void)w;
}

template <int AM, int BMODE, bool TR, int NP, int BN>
__global__ __launch_bounds__(512, 1) void gemm_big_kernel(Args g) {
  constexpr int BM = BIG_BM;
  constexpr int BK = big_bk<NP, AM, BMODE>(), SR = big_sr<BK>(), KS = BK / 16;   // KS: 16-deep MFMA steps per k-tile
  using LA = BigLoader<BM, AM, BK>;
  using LB = BigLoader<BN, BMODE, BK>;
  constexpr int PA = BM * SR, PB = BN * SR;   // one plane
  __shared__ __attribute__((aligned(16))) uint16_t As[2 * NP * PA];
  __shared__ __attribute__((aligned(16))) uint16_t Bs[2 * NP * PB];
  constexpr bool IDX_AHEAD = AM == MN_GATHER || BMODE == MN_GATHER;

  if (g.mdyn) {
    const int64_t m = *g.mdyn;
    g.M = m < g.M ? (m > 0 ? m : 0) : g.M;
  }
  if (g.kdyn) {
    const int64_t k = *g.kdyn;
    g.K = k < g.K ? (k > 0 ? k : 0) : g.K;
    const int64_t kc = (g.K + g.splits - 1) / g.splits;
    g.kchunk = kc > 0 ? (kc + 31) / 32 * 32 : 32;
  }
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, c = lane & 31;
  const int gn = (int)((g.N + BN - 1) / BN);
  const int ntiles = (int)((g.M + BM - 1) / BM) * gn;
  int units = ntiles * g.splits;
  // NR_EPI_SCATTER_ZEROED (destination rows zero on entry, splits == 1): the tiles of the last,
  // partial round of the persistent grid are split along K into `pieces` units whose sums are added
  // atomically, so that round costs 1/pieces of a unit instead of a whole one (a stream-K tail)
  int full = units, rem = 0, pieces = 1;
  int64_t kc_tail = g.kchunk;
  if (g.tail > 1) {
    const int G = (int)gridDim.x;
    const int f = ntiles / G * G, r = ntiles - f;
    if (r > 0 && 2 * r <= G) {
      int p = G / r;
      p = p < g.tail ? p : g.tail;
      const int64_t pmax = g.K / 128;   // >= 8 k-tiles per piece
      p = p < pmax ? p : (int)pmax;
      // pieces through the workspace: one partial tile each, at most tail_cap of them
      if (TR && g.slab && p * r > g.tail_cap) p = g.tail_cap / r;
      if (p > 1) {
        kc_tail = ((g.K + p - 1) / p + 31) / 32 * 32;
        pieces = (int)((g.K + kc_tail - 1) / kc_tail);
      }
    }
    if (pieces > 1) {
      full = f;
      rem = r;
      units = f + r * pieces;
    }
    if (TR && g.slab && blockIdx.x == 0 && tid == 0) {   // the tail reduction's plan (see tail_slab_tr)
      int* hd = reinterpret_cast<int*>(g.slab);
      hd[0] = full; hd[1] = rem; hd[2] = pieces; hd[3] = gn;
    }
  }

  // wave grid: BN = 256 -> 2 (M) x 4 (N) waves of 128x64; BN = 128 -> 4 x 2 waves of 64x64.  Waves
  // w and w + 4 share a SIMD, so at BN = 256 wave w + 4 takes the column block two to the right of
  // wave w's: in a tile cut at half its rows (or columns) every SIMD keeps one wave with live MFMAs.
  // (Such a unit does NOT take half the time -- one wave per SIMD hides less latency -- so the
  // split-K scheduler keeps equal units: balancing them as half-cost measured 362 -> 441 us.)
  constexpr int WN = BN == 256 ? 4 : 2;
  constexpr int TI = (BM / (8 / WN)) / 32, TJ = (BN / WN) / 32;
  const int wm = (w / WN) * (BM / (8 / WN));
  const int wn = (BN == 256 ? (((w & 3) + 2 * (w >> 2)) & 3) : (w % WN)) * (BN / WN);
  f32x16 acc[TI][TJ];
  LA la;
  LB lb;

  // persistent over this block's units (virtual ids blockIdx.x + j * gridDim.x); each unit runs its
  // own two-deep pipeline, so the k-loop carries no unit bookkeeping (a pipeline refill per unit
  // costs one load latency against ~48 k-tiles of MFMAs)
  for (int id = blockIdx.x; id < units; id += gridDim.x) {
    const bool tail_unit = id >= full;
    Unit u;
    int64_t kend;
    if (!tail_unit) {
      u = decode_unit(g, id, full, ntiles, gn, BM, BN);
      if (u.nt <= 0) continue;   // a k-split past a device-resident K
      kend = u.kbeg + g.kchunk < g.K ? u.kbeg + g.kchunk : g.K;
    } else {   // tail: (tile full + j % rem, K piece j / rem)
      const int j = id - full;
      const int tile = full + j % rem;
      u.m0 = (int64_t)(tile / gn) * BM;
      u.n0 = (int64_t)(tile % gn) * BN;
      u.kbeg = (int64_t)(j / rem) * kc_tail;
      kend = u.kbeg + kc_tail < g.K ? u.kbeg + kc_tail : g.K;
      if (kend <= u.kbeg) continue;
    }
    const int nt = (int)((kend - u.kbeg + BK - 1) / BK);
    // a wave whose rows or columns all lie past M / N skips its fragment reads and MFMAs (it still
    // loads, splits and stores its share of the operand tiles)
    const bool live = u.m0 + wm < g.M && u.n0 + wn < g.N;
    // fused bias gradient (slab path, MN-contiguous A): the first column tile's units sum A
    constexpr bool CS_OK = AM == MN_PLAIN && !TR;
    const bool do_cs = CS_OK && g.colsum && g.slab && u.n0 == 0 && !tail_unit;
    float cs[CS_OK ? BigMN<BM, MN_PLAIN, BK>::NC : 1][4];
    if constexpr (CS_OK) {
#pragma unroll
      for (int j = 0; j < BigMN<BM, MN_PLAIN, BK>::NC; ++j) cs[j][0] = cs[j][1] = cs[j][2] = cs[j][3] = 0.f;
    }
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    la.init(g.A, u.m0, g.M, tid);
    lb.init(g.B, u.n0, g.N, tid);
    // k-tile t is loaded into register set t % 2, three tiles ahead of its MFMAs: tile kt+3's loads
    // are issued during k-tile kt and stored to LDS during kt+2 (two MFMA phases of latency cover:
    // the gathered rows come from the Infinity Cache / HBM).  Past the unit's last tile the loads
    // re-read that tile (clamped, never used): the k-tile body stays one basic block.
    auto issue = [&](auto set, int kt) {
      constexpr int S = decltype(set)::value;
      kt = kt < nt ? kt : nt - 1;
      const int64_t k = u.kbeg + (int64_t)kt * BK;
      la.template load<S>(g.A, u.m0, g.M, k, tid);
      lb.template load<S>(g.B, u.n0, g.N, k, tid);
      if (IDX_AHEAD) {   // ids of the set's next tile (kt + 2; clamped to K inside)
        la.template prefetch_idx<S>(g.A, k + 2 * BK, g.K, tid);
        lb.template prefetch_idx<S>(g.B, k + 2 * BK, g.K, tid);
      }
    };
    using S0 = std::integral_constant<int, 0>;
    using S1 = std::integral_constant<int, 1>;
    using LiveT = std::integral_constant<bool, true>;
    using DeadT = std::integral_constant<bool, false>;
    if (IDX_AHEAD) {
      la.template prefetch_idx<0>(g.A, u.kbeg, g.K, tid);
      lb.template prefetch_idx<0>(g.B, u.kbeg, g.K, tid);
      la.template prefetch_idx<1>(g.A, u.kbeg + BK, g.K, tid);
      lb.template prefetch_idx<1>(g.B, u.kbeg + BK, g.K, tid);
    }
    __syncthreads();   // the previous unit's last stage reads are done before stage 0 is rewritten
    issue(S0{}, 0);
    issue(S1{}, 1);
    if constexpr (CS_OK) {
      if (do_cs) la.template add_colsum<0>(cs, tid);
    }
    la.template store<0, NP>(As, tid);
    lb.template store<0, NP>(Bs, tid);
    issue(S0{}, 2);
    __syncthreads();
    // one k-tile (KS MFMA steps of 16): MFMAs from stage st; behind the first row blocks the wave
    // splits k-tile kt+1 (set (kt+1) % 2 = NS) into the other stage, then reuses that set for k-tile
    // kt+3's loads.  The A fragments of row block i+1 are read while row block i's MFMAs run (two
    // fragment register sets), and nothing in a live wave's k-tile branches: the split VALU, the
    // LDS traffic and the MFMAs of one tile form a single scheduling region.  After the unit's last
    // tile the split-stores write the other stage with values nobody reads (the next unit starts
    // behind a barrier and rewrites stage 0).
    // (waves 4-7 splitting behind their last two row blocks instead -- a stagger of the VALU
    // clumps of the two waves on a SIMD -- measured slower: projection fwd 270-280 vs 257-260 µs)
    constexpr int ia = 0, ib = KS == 1 ? 1 : 0;
    auto ktile = [&](auto live_t, auto nset, int kt, int st) {
      constexpr bool LIVE = decltype(live_t)::value;
      constexpr int NS = decltype(nset)::value;
      // the fused column sum runs in every unit of a CS_OK kernel, weighted 0 where the unit does not
      // sum or the register set holds a re-read tile (past the unit's last tile): a runtime test inside
      // the k-tile would split its scheduling region (BERT FFN weight gradient 426 -> 520 us with one)
      const float csf = do_cs && kt + 1 < nt ? 1.f : 0.f;
      (void)csf;
      // interleaved split-stores for bf16x6 on the forward operand pairs (both K-contiguous) and the
      // gathered weight gradient (MN x MN-gathered): one-box A/B (profiles/r04_a_gemm_ab.json, µs)
      // projection fwd 258 -> 248, NRMS weight gradient 292 -> 273, BERT FFN-out 383 -> 376; off for
      // the dgrad pair (K-contiguous A x MN-contiguous B: table dgrad 258 -> 269) and the plain weight
      // gradient (MN x MN: BERT FFN weight gradient 416 -> 447 us, profiles/r04_f_gemm_ab.json)
      constexpr bool ILV = LIVE && NP == 3 && KS == 1 && TJ == 2 && LA::PIECES == 2 && LB::PIECES == 2 &&
                           ((is_kc(AM) && is_kc(BMODE)) || (AM == MN_PLAIN && BMODE == MN_GATHER));
      const uint16_t* a_s = As + st * NP * PA;
      const uint16_t* b_s = Bs + st * NP * PB;
      // after MFMA m (of 12) of row block i: A pieces behind row block ia's MFMAs 2 and 5 (j = 0),
      // B pieces behind row block ib's, the loads of k-tile kt+3 behind its last
      auto ilv_hook = [&](int i, int m) {
        const int piece = m == 2 ? 0 : m == 5 ? 1 : m == 8 ? 2 : 3;
        __builtin_amdgcn_sched_barrier(0);
        if (i == ia && piece < 2) {
          if constexpr (CS_OK) {
            if (piece == 0) la.template add_colsum<NS>(cs, tid, csf);
          }
          la.template store_piece<NS, NP>(As + (st ^ 1) * NP * PA, tid, piece);
        }
        if (i == ib && piece < 2) lb.template store_piece<NS, NP>(Bs + (st ^ 1) * NP * PB, tid, piece);
        if (i == ib && piece == 3) issue(nset, kt + 3);
        __builtin_amdgcn_sched_barrier(0);
      };
      (void)ilv_hook;
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) {
      bf16x8 b[TJ][NP];
      bf16x8 a[2][NP];
      if constexpr (LIVE) {
#pragma unroll
        for (int j = 0; j < TJ; ++j)
#pragma unroll
          for (int p = 0; p < NP; ++p)
            b[j][p] = *reinterpret_cast<const bf16x8*>(b_s + p * PB + (wn + 32 * j + c) * SR + 16 * kk + 8 * h);
#pragma unroll
        for (int p = 0; p < NP; ++p)
          a[0][p] = *reinterpret_cast<const bf16x8*>(a_s + p * PA + (wm + c) * SR + 16 * kk + 8 * h);
      }
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        if constexpr (LIVE) {
          if (i + 1 < TI)
#pragma unroll
            for (int p = 0; p < NP; ++p)
              a[(i + 1) & 1][p] =
                  *reinterpret_cast<const bf16x8*>(a_s + p * PA + (wm + 32 * (i + 1) + c) * SR + 16 * kk + 8 * h);
#pragma unroll
          for (int j = 0; j < TJ; ++j) {
#define NR_MF(X, Y)                                                                                                    \
  acc[i][j] = TR ? __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[j][Y], a[i & 1][X], acc[i][j], 0, 0, 0) \
                 : __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i & 1][X], b[j][Y], acc[i][j], 0, 0, 0)
            if constexpr (ILV) {
              // interleaved: the split-stores of the next stage go in pieces between this row block's
              // MFMAs (a piece's ~22 VALU + its LDS writes behind every third MFMA) instead of as one
              // VALU clump between row blocks, which left the matrix pipe idle when both waves of a
              // SIMD reached it together
              static_assert(NP == 3, "interleave: bf16x6 only");
              NR_MF(2, 0);
              NR_MF(1, 1);
              NR_MF(0, 2);
              ilv_hook(i, 6 * j + 2);
              NR_MF(1, 0);
              NR_MF(0, 1);
              NR_MF(0, 0);
              ilv_hook(i, 6 * j + 5);
            } else {
              if constexpr (NP == 3) {   // smallest terms first
                NR_MF(2, 0);
                NR_MF(1, 1);
                NR_MF(0, 2);
                NR_MF(1, 0);
                NR_MF(0, 1);
              }
              NR_MF(0, 0);
            }
#undef NR_MF
          }
          if constexpr (ILV) continue;
        }
        // split-stores of the next stage: A behind step 0's first row block, B (then the loads of
        // k-tile kt+3 into the freed register set) behind step KS/2's second (KS = 1) or first row block
        if (kk == 0 && i == ia) {
          if constexpr (CS_OK) la.template add_colsum<NS>(cs, tid, csf);
          la.template store<NS, NP>(As + (st ^ 1) * NP * PA, tid);
        }
        if (kk == KS / 2 && i == ib) {
          lb.template store<NS, NP>(Bs + (st ^ 1) * NP * PB, tid);
          issue(nset, kt + 3);
        }
      }
      }
      __syncthreads();   // stage st fully read; stage st^1 fully written
    };
    // unrolled by two: the register sets alternate statically; a wave with no live rows / columns
    // runs the same loads, splits, stores and barriers without fragment reads or MFMAs
    auto kloop = [&](auto live_t) {
      if constexpr (NP == 3) {
        // bf16x6 units always hold an even number of 16-deep k-tiles (the launcher takes K % 32 == 0
        // only; k chunks are multiples of 32): the two-tile body has no branch, so the loop head has
        // one incoming state and hipcc's wait counts at the first split wait for that set's loads
        // only (vmcnt(7..4)), not for the loads issued one tile earlier as well (the merged
        // conditional form waited vmcnt(3..0): one tile of latency cover instead of two)
        for (int kt = 0; kt < nt; kt += 2) {
          ktile(live_t, S1{}, kt, 0);
          ktile(live_t, S0{}, kt + 1, 1);
        }
      } else {
        for (int kt = 0; kt < nt; kt += 2) {
          ktile(live_t, S1{}, kt, 0);
          if (kt + 1 < nt) ktile(live_t, S0{}, kt + 1, 1);
        }
      }
    };
    if (live)
      kloop(LiveT{});
    else
      kloop(DeadT{});
    if (!tail_unit) {
      if constexpr (CS_OK) {
        if (do_cs)
          la.put_colsum(cs, u.m0, g.M,
                        g.slab + (int64_t)g.splits * g.slab_stride + (u.kbeg / g.kchunk) * (g.slab_stride / g.slab_ld),
                        tid);
      }
      if (!TR && g.slab)
        epilogue_slab<TI, TJ>(g, acc, u.m0, u.n0, wm, wn, h, c, g.slab + (u.kbeg / g.kchunk) * g.slab_stride);
      else
        epilogue_any<TR, TI, TJ>(g, acc, u.m0, u.n0, wm, wn, h, c);
    } else if (TR && g.slab) {   // pieces of one tile meet in the workspace, summed by tail_reduce_kernel
      tail_slab_tr<TI, TJ>(acc, wm, wn, h, c, g.slab + TAIL_WS_HDR + (int64_t)(id - full) * 65536);
    } else if (TR) {   // pieces of one tile meet in C: atomic adds into the zeroed destination rows
      static_assert(4 * 32 * 36 * 4 <= 2 * NP * PA * 2 || BN != 256, "tail chunks fit the A image");
      if constexpr (BN == 256 && 4 * 32 * 36 * 4 <= 2 * NP * PB * 2) {
        float* chunk = reinterpret_cast<float*>(w < 4 ? As : Bs) + (w & 3) * 32 * 36;
        tail_scatter_tr<TI, TJ>(g, acc, u.m0, u.n0, wm, wn, h, c, w, lane, chunk);
      } else {
        epilogue_t<NR_EPI_SCATTER, TI, TJ>(g, acc, u.m0, u.n0, wm, wn, h, c, g.vec);
      }
    } else {
      epilogue_cmajor<NR_EPI_SCATTER, TI, TJ>(g, acc, u.m0, u.n0, wm, wn, h, c);
    }
  }
}

template <typename Kern>
int resident_slots_512(Kern k) {
  static int cache[16] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return 0;
  if (cache[dev] == 0) {
    int cus = 0, per = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k, 512, 0) != hipSuccess) return 0;
    cache[dev] = cus * per;
  }
  return cache[dev];
}

template <int AM, int BMODE, bool TR, int NP, int BN>
int launch_big(const Args& g, int splits, hipStream_t s) {
  const int64_t gm = (g.M + BIG_BM - 1) / BIG_BM, gn = (g.N + BN - 1) / BN;
  const int64_t units = gm * gn * splits;
  if (units <= 0) return NR_OK;
  if (units > 0x7fffffff) return NR_EINVAL(0);
  int grid = (int)units;
  const int slots = capped_slots(resident_slots_512(gemm_big_kernel<AM, BMODE, TR, NP, BN>), g.max_cus);
  if (slots > 0 && slots < grid) grid = slots;
  Args a = g;
  a.splits = splits;
  hipLaunchKernelGGL((gemm_big_kernel<AM, BMODE, TR, NP, BN>), dim3((unsigned)grid), dim3(512), 0, s, a);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

// operand-mode dispatch of one (NP, BN); -1 = combination not instantiated
template <int NP, int BN>
int launch_big_modes(const Args& g, int am, int bm, int splits, hipStream_t s) {
  const bool atomic_epi = g.epi == NR_EPI_ATOMIC || g.epi == NR_EPI_SCATTER;
#define NR_BIG(A_, B_, TR_) \
  if (am == A_ && bm == B_ && atomic_epi == !TR_) return launch_big<A_, B_, TR_, NP, BN>(g, splits, s);
  NR_BIG(KC_GATHER, KC_PLAIN, true)    // gathered projection (fwd)
  NR_BIG(KC_PLAIN, KC_PLAIN, true)     // y = x Wᵀ
  NR_BIG(KC_PLAIN, MN_PLAIN, true)     // dgrad (store / scatter-store epilogues)
  NR_BIG(MN_PLAIN, MN_GATHER, false)   // wgrad over gathered rows
  NR_BIG(MN_PLAIN, MN_PLAIN, false)    // wgrad
#undef NR_BIG
  return -1;
}

int launch_big_1_256(const Args& g, int am, int bm, int splits, hipStream_t s);   // gemm_big_*.hip
int launch_big_3_256(const Args& g, int am, int bm, int splits, hipStream_t s);
int launch_big_1_128(const Args& g, int am, int bm, int splits, hipStream_t s);
int launch_big_3_128(const Args& g, int am, int bm, int splits, hipStream_t s);

}  // namespace nrfast
