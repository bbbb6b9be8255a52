// Large-tile bf16 GEMM with the B operand PRE-SPLIT in global memory ("B from global"): the weights of
// the news tower's projection (forward: [Wk; Wv], dgrad: its transpose) and of the BERT dense layers
// are split once per step into their bf16 planes, laid out in MFMA fragment order by nr_split_b, and
// every wave loads its own B fragments straight into registers (one 1-KB coalesced global load per
// fragment and plane, from L2: the weights are small and every CU of an XCD re-reads the same
// column blocks).  Only the big streamed operand A (gathered table rows / dY rows) goes through LDS.
//
// Against the 256 x 256 kernel with both operands in LDS (gemm_big_impl.h) this removes B's split
// (VALU), its LDS stores and its fragment reads, and halves the LDS image, which buys 32-deep k-tiles
// (one barrier per 2 MFMA steps instead of per step) for A.  Waves whose 64 columns lie entirely past
// N (N = 1152 = 4.5 x 256) skip their MFMAs.
#include "gemm_big_impl.h"

namespace nrfast {

constexpr int BG_BK = 32;

template <int AM, int NP>
__global__ __launch_bounds__(512, 1) void gemm_bg_kernel(Args g) {
  constexpr int BM = 256, BN = 256, BK = BG_BK, SR = big_sr<BK>(), KS = BK / 16;
  using LA = BigKC<BM, AM, BK>;
  constexpr int PA = BM * SR;   // one plane of the A image
  __shared__ __attribute__((aligned(16))) uint16_t As[2 * NP * PA];
  if (g.mdyn) {
    const int64_t m = *g.mdyn;
    g.M = m < g.M ? (m > 0 ? m : 0) : g.M;
  }
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, c = lane & 31;
  const int gn = (int)((g.N + BN - 1) / BN);
  const int ntiles = (int)((g.M + BM - 1) / BM) * gn;
  int units = ntiles * g.splits;
  // NR_EPI_SCATTER_ZEROED tail (as gemm_big_kernel): the last partial round's tiles split along K
  int full = units, rem = 0, pieces = 1;
  int64_t kc_tail = g.kchunk;
  if (g.tail > 1) {
    const int G = (int)gridDim.x;
    const int f = ntiles / G * G, r = ntiles - f;
    if (r > 0 && 2 * r <= G) {
      int p = G / r;
      p = p < g.tail ? p : g.tail;
      const int64_t pmax = g.K / 256;   // >= 8 k-tiles per piece
      p = p < pmax ? p : (int)pmax;
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
  }
  // B planes: element (p, n, k) at ((p * NB + n / 32) * KB + k / 16) * 512 + (n % 32) * 16 + k % 16
  const uint16_t* __restrict__ bsrc = reinterpret_cast<const uint16_t*>(g.B.base);
  const int64_t NB = (g.N + 31) / 32, KB = g.B.ld / 16, PS = NB * KB * 512;

  constexpr int TI = 4, TJ = 2;   // 8 waves: 2 (M) x 4 (N), wave tile 128 x 64
  const int wm = (w / 4) * 128, wn = (w % 4) * 64;
  f32x16 acc[TI][TJ];
  LA la;
  for (int id = blockIdx.x; id < units; id += gridDim.x) {
    const bool tail_unit = id >= full;
    Unit u;
    int64_t kend;
    if (!tail_unit) {
      u = decode_unit(g, id, full, ntiles, gn, BM, BN);
      if (u.nt <= 0) continue;
      kend = u.kbeg + g.kchunk < g.K ? u.kbeg + g.kchunk : g.K;
    } else {
      const int j = id - full;
      const int tile = full + j % rem;
      u.m0 = (int64_t)(tile / gn) * BM;
      u.n0 = (int64_t)(tile % gn) * BN;
      u.kbeg = (int64_t)(j / rem) * kc_tail;
      kend = u.kbeg + kc_tail < g.K ? u.kbeg + kc_tail : g.K;
      if (kend <= u.kbeg) continue;
    }
    const int nt = (int)((kend - u.kbeg + BK - 1) / BK);
    const int nsteps = nt * KS;
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    // this wave's B fragment rows (column blocks past N clamp to the last one: discarded)
    const bool live = u.n0 + wn < g.N;
    const uint16_t* bp[TJ];
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      int64_t nb = (u.n0 + wn) / 32 + j;
      nb = nb < NB ? nb : NB - 1;
      bp[j] = bsrc + (nb * KB + u.kbeg / 16) * 512 + c * 16 + 8 * h;
    }
    // B fragments by sub-step q = (MFMA step s, column block j), q = s * TJ + j, in slot q % 2, each
    // loaded one sub-step ahead (half a step of MFMAs covers an L2 hit; two slots instead of a whole
    // step's fragments keep the kernel under 256 VGPRs)
    bf16x8 bq[2][NP];
    auto load_b = [&](auto slot, int q) {
      constexpr int Q = decltype(slot)::value;
      if (!live || q >= nsteps * TJ) return;
      const int s = q / TJ, j = q % TJ;
#pragma unroll
      for (int p = 0; p < NP; ++p)
        bq[Q][p] = *reinterpret_cast<const bf16x8*>(bp[j] + p * PS + (int64_t)s * 512);
    };
    la.init(g.A, u.m0, g.M, tid);
    auto issue = [&](auto set, int kt) {
      constexpr int S = decltype(set)::value;
      la.template load<S>(g.A, u.m0, g.M, u.kbeg + (int64_t)kt * BK, tid);
    };
    using S0 = std::integral_constant<int, 0>;
    using S1 = std::integral_constant<int, 1>;
    // ONE register set for A (the B fragments take the registers of a second): k-tile kt + 1 is
    // split into the other LDS stage during k-tile kt, then the set is reloaded with k-tile kt + 2
    __syncthreads();   // the previous unit's last stage reads are done before stage 0 is rewritten
    issue(S0{}, 0);
    load_b(S0{}, 0);
    la.template store<0, NP>(As, tid);
    if (nt > 1) issue(S0{}, 1);
    __syncthreads();
    auto ktile = [&](int kt, int st) {
      const bool stage_next = kt + 1 < nt;
      const uint16_t* a_s = As + st * NP * PA;
#pragma unroll
      for (int kk = 0; kk < KS; ++kk)
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          // sub-step q = (kt * KS + kk) * TJ + j uses slot (kk * TJ + j) % 2 (KS * TJ even); the next
          // sub-step's fragments go to the other slot
          const int q = (kt * KS + kk) * TJ + j;
          if (((kk * TJ + j) & 1) == 0) load_b(S1{}, q + 1); else load_b(S0{}, q + 1);
#pragma unroll
          for (int i = 0; i < TI; ++i) {
            if (live) {
              bf16x8 a[NP];
#pragma unroll
              for (int p = 0; p < NP; ++p)
                a[p] = *reinterpret_cast<const bf16x8*>(a_s + p * PA + (wm + 32 * i + c) * SR + 16 * kk + 8 * h);
#define NR_MF(X, Y) \
  acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(((kk * TJ + j) & 1) ? bq[1][Y] : bq[0][Y], a[X], acc[i][j], 0, 0, 0)
              if constexpr (NP == 3) {   // smallest terms first
                NR_MF(2, 0);
                NR_MF(1, 1);
                NR_MF(0, 2);
                NR_MF(1, 0);
                NR_MF(0, 1);
              }
              NR_MF(0, 0);
#undef NR_MF
            }
            // behind the k-tile's first row block: split-store of k-tile kt + 1 into the other
            // stage, then the register set's reload with k-tile kt + 2
            if (kk == 0 && j == 0 && i == 0 && stage_next) {
              la.template store<0, NP>(As + (st ^ 1) * NP * PA, tid);
              if (kt + 2 < nt) issue(S0{}, kt + 2);
            }
          }
        }
      __syncthreads();   // stage st fully read; stage st^1 fully written
    };
    for (int kt = 0; kt < nt; kt += 2) {
      ktile(kt, 0);
      if (kt + 1 < nt) ktile(kt + 1, 1);
    }
    if (!tail_unit) {
      epilogue<TI, TJ>(g, acc, u.m0, u.n0, wm, wn, h, c);
    } else {   // pieces of one tile meet in C: atomic adds into the zeroed destination rows
      float* chunk = reinterpret_cast<float*>(As) + w * 32 * 36;
      tail_scatter_tr<TI, TJ>(g, acc, u.m0, u.n0, wm, wn, h, c, w, lane, chunk);
    }
  }
}

template <int AM, int NP>
int launch_bg(const Args& g, int splits, hipStream_t s) {
  const int64_t units = ((g.M + 255) / 256) * ((g.N + 255) / 256) * splits;
  if (units <= 0) return NR_OK;
  if (units > 0x7fffffff) return NR_EINVAL(0);
  int grid = (int)units;
  const int slots = capped_slots(resident_slots_512(gemm_bg_kernel<AM, NP>), g.max_cus);
  if (slots > 0 && slots < grid) grid = slots;
  Args a = g;
  a.splits = splits;
  hipLaunchKernelGGL((gemm_bg_kernel<AM, NP>), dim3((unsigned)grid), dim3(512), 0, s, a);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

// -1: not covered (A must be K-contiguous plain or gathered rows)
int launch_bg_modes(const Args& g, int am, int np, int splits, hipStream_t s) {
  static_assert(4 * 32 * 36 * 8 <= 2 * 1 * 256 * 40 * 2, "tail chunks fit the A image");
  if (am == KC_PLAIN) return np == 3 ? launch_bg<KC_PLAIN, 3>(g, splits, s) : launch_bg<KC_PLAIN, 1>(g, splits, s);
  if (am == KC_GATHER) return np == 3 ? launch_bg<KC_GATHER, 3>(g, splits, s) : launch_bg<KC_GATHER, 1>(g, splits, s);
  return -1;
}

// ---- nr_split_b: fp32 B -> NP bf16 planes in fragment order
template <int NP>
__global__ __launch_bounds__(256) void split_b_kernel(const float* __restrict__ b, int64_t ld, int mn, int64_t N,
                                                      int64_t K, uint16_t* __restrict__ out) {
  // one thread per (n, 4 consecutive k): 4 values -> NP planes of 4 bf16 (8 B each)
  const int64_t NB = (N + 31) / 32, KB = K / 16, PS = NB * KB * 512;
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;   // over NB*32 rows x K/4 quads
  const int64_t kq = K / 4;
  if (q >= NB * 32 * kq) return;
  const int64_t n = q / kq, k = (q - n * kq) * 4;
  float x[4] = {0.f, 0.f, 0.f, 0.f};
  if (n < N) {
    if (!mn) {
      const float4 v = *reinterpret_cast<const float4*>(b + n * ld + k);
      x[0] = v.x; x[1] = v.y; x[2] = v.z; x[3] = v.w;
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) x[u] = b[(k + u) * ld + n];
    }
  }
  const int64_t off = ((n / 32) * KB + k / 16) * 512 + (n % 32) * 16 + k % 16;
  if constexpr (NP == 1) {
    *reinterpret_cast<uint2*>(out + off) = hi4(x[0], x[1], x[2], x[3]);
  } else {
    uint2 p0, p1, p2;
    split4(x[0], x[1], x[2], x[3], p0, p1, p2);
    *reinterpret_cast<uint2*>(out + off) = p0;
    *reinterpret_cast<uint2*>(out + PS + off) = p1;
    *reinterpret_cast<uint2*>(out + 2 * PS + off) = p2;
  }
}

}  // namespace nrfast

extern "C" int64_t nr_split_b_elems(int64_t N, int64_t K, int32_t np) {
  if (N < 0 || K < 0 || (K % 32) || (np != 1 && np != 3)) return -1;
  return (int64_t)np * ((N + 31) / 32) * (K / 16) * 512;
}

extern "C" int nr_split_b(const float* b, int64_t ld, int32_t layout, int64_t N, int64_t K, int32_t np,
                          uint16_t* out, hipStream_t stream) {
  using namespace nrfast;
  if (N < 0 || K < 0 || (K % 32) || (np != 1 && np != 3)) return NR_EINVAL(0);
  if (layout != NR_KCONTIG && layout != NR_MNCONTIG) return NR_EINVAL(2);
  if (N == 0 || K == 0) return NR_OK;
  if (!b || !out) return NR_EINVAL(1);
  if (layout == NR_KCONTIG && ((ld & 3) || (reinterpret_cast<uintptr_t>(b) & 15))) return NR_EINVAL(1);
  if ((reinterpret_cast<uintptr_t>(out) & 7)) return NR_EINVAL(6);
  const int64_t total = ((N + 31) / 32) * 32 * (K / 4);
  const dim3 grid((unsigned)((total + 255) / 256));
  const int mn = layout == NR_MNCONTIG;
  if (np == 3)
    hipLaunchKernelGGL(split_b_kernel<3>, grid, dim3(256), 0, stream, b, ld, mn, N, K, out);
  else
    hipLaunchKernelGGL(split_b_kernel<1>, grid, dim3(256), 0, stream, b, ld, mn, N, K, out);
  NR_LAUNCH_CHECK();
  return NR_OK;
}
