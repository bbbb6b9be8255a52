// The exact-f32 fast GEMM kernel (persistent, two-deep pipelined) and its launchers, included by
// gemm_fast.hip (128x128 tiles + the entry point) and gemm_fast64.hip (64x64 tiles) so the
// instantiations compile in parallel.
#pragma once
#include "gemm_fast_common.h"

namespace nrfast {


// Persistent GEMM: a grid of (resident blocks) walks the units with stride gridDim.x, and the
// k-loop runs over the flattened (unit, k-tile) sequence.  Two-deep pipeline per block: while
// the MFMAs consume k-tile P from LDS, tile P+1 sits in registers and is written to the other
// LDS buffer after the first quarter of P's MFMAs, and the global loads of P+2 are issued right
// behind that write — so a load has a whole iteration to land, the LDS write never waits, and
// each iteration ends in a bare barrier.  Unit boundaries are invisible to the pipeline: the
// next unit's first tiles load during the current unit's last ones, and the finished unit's
// epilogue stores go out behind them.  A grid of `units` blocks is the plain one-tile-per-block
// kernel.
template <int BM, int BN, int AM, int BMODE, bool TR>
__global__ __launch_bounds__(256, 2) void gemm_fast_kernel(Args g) {
  using LA = Loader<BM, AM>;
  using LB = Loader<BN, BMODE>;
  __shared__ __attribute__((aligned(16))) float As[2][LA::LDS_FLOATS];
  __shared__ __attribute__((aligned(16))) float Bs[2][LB::LDS_FLOATS];
  constexpr bool IDX_AHEAD = AM == MN_GATHER || BMODE == MN_GATHER;

  // device-resident extents (row counts produced on the GPU, e.g. nr_unique_rows): the host
  // sizes were upper bounds for the grid
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

  // first non-empty unit at or after virtual id `id` in this block's sequence (a split past a
  // device-resident K is empty), or `units`
  auto skip_empty = [&](int id, Unit& u) -> int {
    for (; id < units; id += G) {
      u = decode_unit(g, id, units, ntiles, gn, BM, BN);
      if (u.nt > 0) return id;
    }
    return units;
  };
  // cursor advance: false when the block's sequence is exhausted
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
  auto peek_k = [&](const Cursor& p) -> int64_t {   // k of the position after p, or -1
    if (p.kt + 1 < p.u.nt) return kof(p) + 32;
    Unit u;
    return skip_empty(p.id + G, u) < units ? u.kbeg : -1;
  };

  Cursor cp;   // compute position
  cp.kt = 0;
  cp.id = skip_empty(blockIdx.x, cp.u);
  if (cp.id >= units) return;

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
  Cursor lp = cp;   // load position
  la.init(g.A, lp.u.m0, g.M, tid);
  lb.init(g.B, lp.u.n0, g.N, tid);
  auto issue = [&](const Cursor& p) {
    const int64_t k = kof(p);
    la.load(g.A, p.u.m0, g.M, k, tid);
    lb.load(g.B, p.u.n0, g.N, k, tid);
    if (IDX_AHEAD) {   // token ids of the position after p, one load ahead of its data
      const int64_t pk = peek_k(p);
      if (pk >= 0) {
        la.prefetch_idx(g.A, pk, g.K, tid);
        lb.prefetch_idx(g.B, pk, g.K, tid);
      }
    }
  };
  auto step_load = [&]() -> bool {   // move lp one position and issue its loads
    const int old = lp.id;
    if (!advance(lp)) return false;
    if (lp.id != old) {
      la.init(g.A, lp.u.m0, g.M, tid);
      lb.init(g.B, lp.u.n0, g.N, tid);
    }
    issue(lp);
    return true;
  };

  // prologue: P0 -> LDS[0], P1 -> registers
  if (IDX_AHEAD) {
    la.prefetch_idx(g.A, kof(lp), g.K, tid);
    lb.prefetch_idx(g.B, kof(lp), g.K, tid);
  }
  issue(lp);
  la.store(As[0], tid);
  lb.store(Bs[0], tid);
  bool staged = step_load();   // registers hold the position after cp
  __syncthreads();

  bool pending = false;
  int64_t pm0 = 0, pn0 = 0;
  int buf = 0;
  for (;;) {
    if (pending) {   // previous unit's output, behind this unit's first loads
      epilogue_any<TR, TI, TJ>(g, acc, pm0, pn0, wm, wn, h, c);
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
      pending = false;
    }
    const float* a_s = As[buf];
    const float* b_s = Bs[buf];
    const bool had_staged = staged;
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
          acc[i][j] = TR ? __builtin_amdgcn_mfma_f32_32x32x2f32(b[j].x, a[i].x, acc[i][j], 0, 0, 0)
                         : __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].x, b[j].x, acc[i][j], 0, 0, 0);
          acc[i][j] = TR ? __builtin_amdgcn_mfma_f32_32x32x2f32(b[j].y, a[i].y, acc[i][j], 0, 0, 0)
                         : __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].y, b[j].y, acc[i][j], 0, 0, 0);
          acc[i][j] = TR ? __builtin_amdgcn_mfma_f32_32x32x2f32(b[j].z, a[i].z, acc[i][j], 0, 0, 0)
                         : __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].z, b[j].z, acc[i][j], 0, 0, 0);
          acc[i][j] = TR ? __builtin_amdgcn_mfma_f32_32x32x2f32(b[j].w, a[i].w, acc[i][j], 0, 0, 0)
                         : __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].w, b[j].w, acc[i][j], 0, 0, 0);
        }
      if (q == 0 && had_staged) {   // publish P+1 (its buffer's readers passed the last barrier)
        la.store(As[buf ^ 1], tid);
        lb.store(Bs[buf ^ 1], tid);
        staged = step_load();       // and start P+2
      }
    }
    __syncthreads();
    buf ^= 1;
    const int old = cp.id;
    const int64_t om0 = cp.u.m0, on0 = cp.u.n0;
    if (!had_staged) break;         // cp was the block's last position
    advance(cp);
    if (cp.id != old) {
      pending = true;
      pm0 = om0;
      pn0 = on0;
    }
  }
  epilogue_any<TR, TI, TJ>(g, acc, cp.u.m0, cp.u.n0, wm, wn, h, c);
}

template <int BM, int BN, int AM, int BMODE, bool TR>
int launch(const Args& g, int splits, hipStream_t s) {
  const int64_t gm = (g.M + BM - 1) / BM, gn = (g.N + BN - 1) / BN;
  const int64_t units = gm * gn * splits;
  if (units <= 0) return NR_OK;
  if (units > 0x7fffffff) return NR_EINVAL(0);
  int grid = (int)units;
  {
    const int slots = capped_slots(resident_slots(gemm_fast_kernel<BM, BN, AM, BMODE, TR>), g.max_cus);
    if (slots > 0 && slots < grid) grid = slots;
  }
  Args a = g;
  a.splits = splits;
  hipLaunchKernelGGL((gemm_fast_kernel<BM, BN, AM, BMODE, TR>), dim3((unsigned)grid), dim3(256), 0, s, a);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

template <int BM, int BN>
int launch_modes(const Args& g, int am, int bm, int splits, int prec, hipStream_t s) {
  if (BM == 128 && BN == 128 && prec != NR_GEMM_F32) {
    const int rc = launch_split_modes(g, am, bm, splits, prec == NR_GEMM_BF16 ? 1 : 3, s);
    if (rc != -1) return rc;
  }
#define NR_AB(A_, B_, TR_) \
  if (am == A_ && bm == B_ && atomic_epi == !TR_) return launch<BM, BN, A_, B_, TR_>(g, splits, s);
  // transposed accumulators (float4 stores) for store epilogues, C-major for atomic ones
  const bool atomic_epi = g.epi == NR_EPI_ATOMIC || g.epi == NR_EPI_SCATTER;
  NR_AB(KC_GATHER, KC_PLAIN, true)    // fused gather + projection (fwd)
  NR_AB(KC_CONV3, KC_PLAIN, true)     // conv as K = 3E GEMM (fwd)
  NR_AB(KC_PLAIN, KC_PLAIN, true)     // plain y = x Wᵀ
  NR_AB(KC_PLAIN, MN_PLAIN, true)     // dgrad dx = dy W
  NR_AB(KC_PLAIN, MN_PLAIN, false)    // dgrad scattered into the word-table gradient
  NR_AB(MN_PLAIN, MN_GATHER, false)   // wgrad dW = dyᵀ table[ids]
  NR_AB(MN_PLAIN, MN_CONV3, false)    // conv wgrad
  NR_AB(MN_PLAIN, MN_PLAIN, false)    // wgrad dW = dyᵀ x
#undef NR_AB
  return -1;
}

}  // namespace nrfast
