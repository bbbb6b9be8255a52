// bf16 matrix-core GEMM kernels (NR_GEMM_BF16X6: NP = 3 planes, six products; NR_GEMM_BF16: NP = 1,
// one product), included by the gemm_split_*.hip translation units so the instantiations compile in
// parallel.  Shared code: gemm_fast_common.h.
#pragma once
#include <type_traits>

#include "gemm_fast_common.h"

namespace nrfast {

// bf16x6 form of gemm_fast_kernel (128x128 tiles, the same persistent two-deep pipeline and
// epilogues): the loaders split each fp32 element into three bf16 planes as they publish a
// k-tile to LDS (K-contiguous operands as loaded, MN-contiguous ones through a 4x4 register
// transpose), and each 16-deep k-step runs six v_mfma_f32_32x32x16_bf16 per 32x32 output tile,
// smallest terms first.  The accumulators have the f32 MFMA's C/D layout, so the epilogues are
// shared.  One LDS image (60 KiB) so two workgroups share a CU: tile P+1 waits in registers while
// P computes, is published between two barriers, and P+2's loads go out right behind it.
// NP = 1 (bf16 arithmetic): the same pipeline with one plane per operand and one MFMA per
// 32x32 tile and k-step (fp32 operands rounded to bf16 on the way to LDS, fp32 accumulation).
template <int AM, int BMODE, bool TR, int NP>
__global__ __launch_bounds__(256, 2) void gemm_split_kernel(Args g) {
  using LA = typename std::conditional<is_kc(AM), Loader<128, AM>, MNBlk<AM>>::type;
  using LB = typename std::conditional<is_kc(BMODE), Loader<128, BMODE>, MNBlk<BMODE>>::type;
  constexpr int BM = 128, BN = 128;
  __shared__ __attribute__((aligned(16))) uint16_t As[NP * SPL];
  __shared__ __attribute__((aligned(16))) uint16_t Bs[NP * SPL];
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
  const int units = ntiles * g.splits;
  const int G = gridDim.x;

  auto skip_empty = [&](int id, Unit& u) -> int {
    for (; id < units; id += G) {
      u = decode_unit(g, id, units, ntiles, gn, BM, BN);
      if (u.nt > 0) return id;
    }
    return units;
  };
  auto advance = [&](Cursor& p) -> bool {
    if (p.kt + 1 < p.u.nt) { ++p.kt; return true; }
    Unit u;
    const int nid = skip_empty(p.id + G, u);
    if (nid >= units) return false;
    p.id = nid;
    p.kt = 0;
    p.u = u;
    return true;
  };
  auto kof = [](const Cursor& p) -> int64_t { return p.u.kbeg + (int64_t)p.kt * 32; };
  auto peek_k = [&](const Cursor& p) -> int64_t {
    if (p.kt + 1 < p.u.nt) return kof(p) + 32;
    Unit u;
    return skip_empty(p.id + G, u) < units ? u.kbeg : -1;
  };

  Cursor cp;
  cp.kt = 0;
  cp.id = skip_empty(blockIdx.x, cp.u);
  if (cp.id >= units) return;

  constexpr int TI = 2, TJ = 2;
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
  Cursor lp = cp;
  la.init(g.A, lp.u.m0, g.M, tid);
  lb.init(g.B, lp.u.n0, g.N, tid);
  auto issue = [&](const Cursor& p) {
    const int64_t k = kof(p);
    la.load(g.A, p.u.m0, g.M, k, tid);
    lb.load(g.B, p.u.n0, g.N, k, tid);
    if (IDX_AHEAD) {
      const int64_t pk = peek_k(p);
      if (pk >= 0) {
        la.prefetch_idx(g.A, pk, g.K, tid);
        lb.prefetch_idx(g.B, pk, g.K, tid);
      }
    }
  };
  auto step_load = [&]() -> bool {
    const int old = lp.id;
    if (!advance(lp)) return false;
    if (lp.id != old) {
      la.init(g.A, lp.u.m0, g.M, tid);
      lb.init(g.B, lp.u.n0, g.N, tid);
    }
    issue(lp);
    return true;
  };

  if (IDX_AHEAD) {
    la.prefetch_idx(g.A, kof(lp), g.K, tid);
    lb.prefetch_idx(g.B, kof(lp), g.K, tid);
  }
  issue(lp);
  la.template store_split<NP>(As, tid);
  lb.template store_split<NP>(Bs, tid);
  bool staged = step_load();
  __syncthreads();

  bool pending = false;
  int64_t pm0 = 0, pn0 = 0;
  for (;;) {
    if (pending) {
      epilogue_any<TR, TI, TJ>(g, acc, pm0, pn0, wm, wn, h, c);
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
      pending = false;
    }
    const uint16_t* a_s = As;
    const uint16_t* b_s = Bs;
    const bool had_staged = staged;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 a[TI][NP], b[TJ][NP];
      const int ko = 16 * s + 8 * h;
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int p = 0; p < NP; ++p)
          a[i][p] = *reinterpret_cast<const bf16x8*>(a_s + p * SPL + (wm + 32 * i + c) * SROW + ko);
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int p = 0; p < NP; ++p)
          b[j][p] = *reinterpret_cast<const bf16x8*>(b_s + p * SPL + (wn + 32 * j + c) * SROW + ko);
#define NR_MF(X, Y)                                                                              \
  acc[i][j] = TR ? __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[j][Y], a[i][X], acc[i][j], 0, 0, 0) \
                 : __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][X], b[j][Y], acc[i][j], 0, 0, 0)
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
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
    __syncthreads();                // every wave is done reading P
    const int old = cp.id;
    const int64_t om0 = cp.u.m0, on0 = cp.u.n0;
    if (!had_staged) break;
    la.template store_split<NP>(As, tid);   // publish P+1 (its loads landed during P's MFMAs)
    lb.template store_split<NP>(Bs, tid);
    staged = step_load();           // and start P+2
    __syncthreads();
    advance(cp);
    if (cp.id != old) {
      pending = true;
      pm0 = om0;
      pn0 = on0;
    }
  }
  epilogue_any<TR, TI, TJ>(g, acc, cp.u.m0, cp.u.n0, wm, wn, h, c);
}

template <int AM, int BMODE, bool TR, int NP>
int launch_split(const Args& g, int splits, hipStream_t s) {
  const int64_t gm = (g.M + 127) / 128, gn = (g.N + 127) / 128;
  const int64_t units = gm * gn * splits;
  if (units <= 0) return NR_OK;
  if (units > 0x7fffffff) return NR_EINVAL(0);
  int grid = (int)units;
  {
    const int slots = capped_slots(resident_slots(gemm_split_kernel<AM, BMODE, TR, NP>), g.max_cus);
    if (slots > 0 && slots < grid) grid = slots;
  }
  Args a = g;
  a.splits = splits;
  hipLaunchKernelGGL((gemm_split_kernel<AM, BMODE, TR, NP>), dim3((unsigned)grid), dim3(256), 0, s, a);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

// K-contiguous A operand (projections, dgrads)
template <int NP>
int launch_split_kc(const Args& g, int am, int bm, int splits, hipStream_t s) {
  const bool atomic_epi = g.epi == NR_EPI_ATOMIC || g.epi == NR_EPI_SCATTER;
#define NR_SAB(A_, B_, TR_) \
  if (am == A_ && bm == B_ && atomic_epi == !TR_) return launch_split<A_, B_, TR_, NP>(g, splits, s);
  NR_SAB(KC_GATHER, KC_PLAIN, true)
  NR_SAB(KC_CONV3, KC_PLAIN, true)
  NR_SAB(KC_PLAIN, KC_PLAIN, true)
  NR_SAB(KC_PLAIN, MN_PLAIN, true)
  NR_SAB(KC_PLAIN, MN_PLAIN, false)
#undef NR_SAB
  return -1;
}

// MN-contiguous A operand (weight gradients)
template <int NP>
int launch_split_mn(const Args& g, int am, int bm, int splits, hipStream_t s) {
  const bool atomic_epi = g.epi == NR_EPI_ATOMIC || g.epi == NR_EPI_SCATTER;
  if (!atomic_epi || am != MN_PLAIN) return -1;
  if (bm == MN_GATHER) return launch_split<MN_PLAIN, MN_GATHER, false, NP>(g, splits, s);
  if (bm == MN_PLAIN) return launch_split<MN_PLAIN, MN_PLAIN, false, NP>(g, splits, s);
  if (bm == MN_CONV3 && g.B.seg % 128 == 0) return launch_split<MN_PLAIN, MN_CONV3, false, NP>(g, splits, s);
  return -1;
}

// one translation unit per (operand family, plane count): gemm_split_{kc,mn}{1,3}.hip
int launch_split_kc1(const Args& g, int am, int bm, int splits, hipStream_t s);
int launch_split_kc3(const Args& g, int am, int bm, int splits, hipStream_t s);
int launch_split_mn1(const Args& g, int am, int bm, int splits, hipStream_t s);
int launch_split_mn3(const Args& g, int am, int bm, int splits, hipStream_t s);

}  // namespace nrfast
