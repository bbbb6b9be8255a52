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
#include <stdlib.h>

#include "gemm_fast.h"

#include "gemm_fast_impl.h"

namespace nrfast {
int launch_modes64(const Args& g, int am, int bm, int splits, hipStream_t s);   // gemm_fast64.hip
int launch_big_1_256(const Args& g, int am, int bm, int splits, hipStream_t s);   // gemm_big_*.hip
int launch_big_3_256(const Args& g, int am, int bm, int splits, hipStream_t s);
int launch_big_1_128(const Args& g, int am, int bm, int splits, hipStream_t s);
int launch_big_3_128(const Args& g, int am, int bm, int splits, hipStream_t s);

// Large-tile (256 x BN) bf16 kernel choice: 0 = stay on the 128x128 kernel; 256 x 256 tiles unless
// their units fill the 256 CUs clearly worse ("round efficiency" = units / (256 * rounds), times the useful fraction
// of padded columns) than the 128x128 kernel's at two workgroups per CU.
// Split-K callers (atomic epilogues) are re-split for the chosen tile, so they always fill the chip.
double round_eff(int64_t units, int64_t slots) {
  if (units <= 0) return 0.0;
  const int64_t rounds = (units + slots - 1) / slots;
  return (double)units / (double)(rounds * slots);
}

int big_bn(int64_t M, int64_t N, int64_t K, int splits, bool resplit, bool m_dyn, int kmin) {
  if (N < 128) return 0;
  // a short contraction (K < kmin) does not amortise the per-unit pipeline fill
  if (!resplit && K < kmin) return 0;
  const int64_t gm = (M + 255) / 256;
  if (!resplit && gm * splits < 8) return 0;
  if (resplit) return (N % 256 == 0 || N >= 1024) ? 256 : 128;
  // padded-N MFMA work counts against a tile width too; measured on the step's shapes, the
  // 256 x 256 core is ~15 % faster per unit of work than the 128 x 128 kernel, 256 x 128 is not
  const double e256 = round_eff(gm * ((N + 255) / 256) * splits, 256) * (double)N / (double)((N + 255) / 256 * 256);
  const double e_old = round_eff(((M + 127) / 128) * ((N + 127) / 128) * splits, 512) * (double)N /
                       (double)((N + 127) / 128 * 128);
  // device-resident M (distinct-row counts): the host M is only a bound and the persistent grid
  // absorbs the actual count -- the big tiles for wide N, else the round efficiencies at the bound
  // (the CNN tap projection, N = 480: 141 -> see DESIGN §4.1)
  if (m_dyn) return (N >= 1024 || e256 >= 0.87 * e_old) ? 256 : 0;
  return e256 >= 0.87 * e_old ? 256 : 0;
}
// Split-K slabs -> C: C[m][n] += sum over the valid splits of slab[s][m][n], in split order
// (deterministic).  The valid split count and row count follow the GEMM kernel's own reading of
// the device-resident K / M (a split whose k range starts past the device K wrote nothing).
__global__ __launch_bounds__(256) void splitk_reduce_kernel(float* __restrict__ C, int64_t ldc,
                                                            const float* __restrict__ slab, int64_t ld,
                                                            int64_t stride, int splits, int64_t M, int64_t N,
                                                            int64_t K, int64_t kchunk, const int32_t* mdyn,
                                                            const int32_t* kdyn, int vec, float* __restrict__ colsum) {
  int64_t m_eff = M;
  if (mdyn) {
    const int64_t m = *mdyn;
    m_eff = m < M ? (m > 0 ? m : 0) : M;
  }
  int ns = splits;
  if (kdyn) {
    int64_t k = *kdyn;
    k = k < K ? (k > 0 ? k : 0) : K;
    const int64_t kc = (k + splits - 1) / splits;
    const int64_t kch = kc > 0 ? (kc + 31) / 32 * 32 : 32;
    ns = (int)((k + kch - 1) / kch);
  } else {
    ns = (int)((K + kchunk - 1) / kchunk);
  }
  ns = ns < splits ? ns : splits;
  const int64_t n4 = (N + 3) / 4, total = m_eff * n4;
  if (colsum) {   // the fused bias gradient: per-split column sums after the partial tiles
    const float* cs = slab + (int64_t)splits * stride;
    const int64_t mh = stride / ld;
    for (int64_t m = (int64_t)blockIdx.x * 256 + threadIdx.x; m < m_eff; m += (int64_t)gridDim.x * 256) {
      float a = colsum[m];
      for (int sp = 0; sp < ns; ++sp) a += cs[sp * mh + m];
      colsum[m] = a;
    }
  }
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t m = i / n4, n = 4 * (i - m * n4);
    const float* s = slab + m * ld + n;
    float* c = C + m * ldc + n;
    if (vec && n + 3 < N) {
      float4 a = *reinterpret_cast<const float4*>(c);
#pragma unroll 4
      for (int sp = 0; sp < ns; ++sp) {
        const float4 x = *reinterpret_cast<const float4*>(s + sp * stride);
        a.x += x.x; a.y += x.y; a.z += x.z; a.w += x.w;
      }
      *reinterpret_cast<float4*>(c) = a;
    } else {
      for (int e = 0; e < 4 && n + e < N; ++e) {
        float a = c[e];
        for (int sp = 0; sp < ns; ++sp) a += s[sp * stride + e];
        c[e] = a;
      }
    }
  }
}

// The big kernel's stream-K tail through its workspace (tail_slab_tr): every tail tile's pieces added
// in piece order (deterministic) and stored to the tile's distinct destination rows (rows[m]; pad_row
// and rows past the device-resident M skipped), the plan read from the header the GEMM wrote.
__global__ __launch_bounds__(256) void tail_reduce_kernel(float* __restrict__ C, int64_t ldc,
                                                          const float* __restrict__ ws, const int64_t* __restrict__ rows,
                                                          int64_t pad_row, int64_t M, const int32_t* mdyn, int64_t N,
                                                          int vec) {
  const int* hd = reinterpret_cast<const int*>(ws);
  const int full = hd[0], rem = hd[1], pieces = hd[2], gn = hd[3];
  if (pieces <= 1 || rem <= 0 || gn <= 0) return;
  int64_t m_eff = M;
  if (mdyn) {
    const int64_t m = *mdyn;
    m_eff = m < M ? (m > 0 ? m : 0) : M;
  }
  const float* part = ws + TAIL_WS_HDR;
  const int64_t total = (int64_t)rem * 256 * 64;   // float4 of the rem tail tiles
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    const int t = (int)(e >> 14), w = (int)(e & 16383), r = w >> 6, c4 = w & 63;
    const int tile = full + t;
    const int64_t m = (int64_t)(tile / gn) * 256 + r, n = (int64_t)(tile % gn) * 256 + 4 * c4;
    if (m >= m_eff || n >= N) continue;
    const int64_t tok = rows[m];
    if (tok == pad_row) continue;
    const float* s = part + (int64_t)t * 65536 + r * 256 + 4 * c4;
    float4 a = *reinterpret_cast<const float4*>(s);
    for (int q = 1; q < pieces; ++q) {
      const float4 x = *reinterpret_cast<const float4*>(s + (int64_t)q * rem * 65536);
      a.x += x.x; a.y += x.y; a.z += x.z; a.w += x.w;
    }
    float* c = C + tok * ldc + n;
    if (vec && n + 3 < N) {
      *reinterpret_cast<float4*>(c) = a;
    } else {
      const float v[4] = {a.x, a.y, a.z, a.w};
      for (int u = 0; u < 4 && n + u < N; ++u) c[u] = v[u];
    }
  }
}

}  // namespace nrfast

// Elements of nr_gemm_f32_ws' split-K workspace that serve any shape: one round of 256 x 256
// partial tiles over the device's CUs (the big kernel re-splits a split-K contraction to one unit
// per CU), plus row padding and the per-split column sums.
extern "C" int64_t nr_gemm_splitk_workspace(void) {
  const int cus = nrfast::device_cus();
  return (int64_t)(cus > 0 ? cus : 256) * 256 * 261;
}


// Returns -1 if the shape/operands are not eligible (the caller falls back), else a status.
int nr_gemm_fast(int64_t M, int64_t N, int64_t K, const nr_operand* A, const nr_operand* B, float* C,
                 int64_t ldc, const float* bias, int32_t epilogue, const nr_operand* c_rows, int64_t pad_row,
                 int32_t split_k, int bm, int bn, const int32_t* m_dev, const int32_t* k_dev, int32_t prec,
                 int32_t max_cus, float* work, int64_t work_elems, float* colsum, int32_t* colsum_folded,
                 hipStream_t stream) {
  using namespace nrfast;
  if (K <= 0) return -1;
  // NR_EPI_SCATTER_ZEROED = NR_EPI_SCATTER_STORE whose destination rows are zero on entry: the big
  // kernel may then split the K of its last partial round of tiles (atomic adds of the pieces)
  const bool zeroed = epilogue == NR_EPI_SCATTER_ZEROED;
  if (zeroed) epilogue = NR_EPI_SCATTER_STORE;
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
  if (epilogue == NR_EPI_SCATTER_STORE && (!c_rows || c_rows->map != NR_ROWS_GATHER || !c_rows->rows)) return -1;
  if (epilogue == NR_EPI_SCATTER && c_rows && c_rows->map == NR_ROWS_CONV3 && c_rows->seq_len == 1) return -1;
  g.C = C; g.ldc = ldc; g.bias = bias; g.epi = epilogue; g.pad_row = pad_row;
  g.mdyn = m_dev; g.kdyn = k_dev; g.splits = 1; g.tail = 0; g.max_cus = max_cus > 0 ? max_cus : 0;
  {
    auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    bool v = N % 4 == 0 && ldc % 4 == 0 && al16(C) && (!bias || al16(bias));
    if (epilogue == NR_EPI_ACCUM_GATE || epilogue == NR_EPI_STORE_GELU || epilogue == NR_EPI_GELU_GRAD)
      v = v && c_rows && c_rows->ld % 4 == 0 && al16(c_rows->data);
    g.vec = v ? 1 : 0;
  }
  g.kchunk = (K + split_k - 1) / split_k;
  g.kchunk = (g.kchunk + 31) / 32 * 32;
  if (g.kchunk == 0) g.kchunk = 32;
  const int splits = (int)((K + g.kchunk - 1) / g.kchunk) > 0 ? (int)((K + g.kchunk - 1) / g.kchunk) : 1;
  if (bm == 128 && bn == 128 && prec != NR_GEMM_F32) {
    const bool resplit = split_k > 1 && (epilogue == NR_EPI_ATOMIC || epilogue == NR_EPI_SCATTER);
    // shortest contraction the big kernel takes: 512 (32 k-tiles of MFMAs per unit fill), in bf16 too
    // (A/B: the CNN table dgrad, K = 480, ran 94 us on the 128x128 kernel and 114 us on the big one)
    // (re-measured in round 4 on the k-contiguous CNN dgrad, bf16: 59 us here, 95 us with kmin = 480,
    // profiles/r04_h_gemm_ab.json)
    const int kmin = 512;
    // the stream-K tail through the workspace (bf16x6, below) makes the big kernel pay for contractions
    // down to 256 too: the CNN table dgrad (K = 480) left the 128 x 128 kernel with it
    const bool ws_tail = zeroed && prec == NR_GEMM_BF16X6 && work != nullptr;
    const int kmin_t = ws_tail ? 256 : kmin;
    const bool tailed = zeroed && splits == 1 && K >= kmin_t && N >= 256 && big_bn(M, N, K, 1, false, false, kmin_t) >= 0;
    // bf16 split-K (atomic) launches take the big kernel too: its fewer, larger units halve the operand
    // re-reads and keep three k-tiles of loads in flight (CNN conv weight gradient 200 -> 138 us)
    const int bb = big_bn(M, N, K, splits, resplit, m_dev != nullptr, kmin);
    // the bf16x6 big kernel runs its k-loop two 16-deep k-tiles per iteration with no branch: every
    // unit's k range must be a multiple of 32 (k chunks are; K must be)
    const int BN = prec == NR_GEMM_BF16X6 && K % 32 != 0 ? 0 : (tailed ? 256 : (bb > 0 ? bb : 0));
    if (BN) {
      Args gb = g;
      if (tailed) gb.tail = 16;
      int sp = splits;
      if (resplit) {
        // re-split for 256 x BN tiles: one wave of units over the CUs it may use, >= 512 k per split
        const int64_t tiles = ((M + 255) / 256) * ((N + BN - 1) / BN);
        const int cus = g.max_cus > 0 ? g.max_cus : 256;
        int64_t want = cus / (tiles > 0 ? tiles : 1);
        if (want > K / 512) want = K / 512;
        if (want > 64) want = 64;
        if (want < 1) want = 1;
        gb.kchunk = ((K + want - 1) / want + 31) / 32 * 32;
        sp = (int)((K + gb.kchunk - 1) / gb.kchunk);
      }
      // split-K partial tiles through a workspace (plain stores + one reduction launch) when the caller
      // gave one: a round of 256 fp32 atomic tiles costs ~50 us at the chip's ~1.3 TB/s atomic rate
      const int64_t sld = (N + 3) & ~int64_t(3);
      const bool slab = epilogue == NR_EPI_ATOMIC && sp > 1 && work &&
                        work_elems >= (int64_t)sp * M * sld + (colsum ? (int64_t)sp * M : 0) &&
                        (reinterpret_cast<uintptr_t>(work) & 15) == 0;
      const bool fold = slab && colsum && am == MN_PLAIN;
      // the stream-K tail's pieces through the workspace too (tail_slab_tr / tail_reduce_kernel): one
      // 256 x 256 partial tile per tail unit; the kernel's plan keeps the pieces within the tiles the
      // workspace holds (Args::tail_cap), so a grid of more than one workgroup per CU cannot overrun it
      // (bf16x6: one 147 KB workgroup per CU; the bf16 kernel keeps the atomic tail)
      const int cus = device_cus();
      const int64_t cap_tiles = work_elems > TAIL_WS_HDR ? (work_elems - TAIL_WS_HDR) / 65536 : 0;
      const bool tail_ws = tailed && prec == NR_GEMM_BF16X6 && work && cus > 0 && cap_tiles >= cus &&
                           (reinterpret_cast<uintptr_t>(work) & 15) == 0;
      if (tail_ws) {
        gb.slab = work;
        gb.tail_cap = (int)(cap_tiles < 0x7fffffff ? cap_tiles : 0x7fffffff);
      }
      if (slab) {
        gb.slab = work;
        gb.slab_ld = sld;
        gb.slab_stride = M * sld;
        gb.colsum = fold ? colsum : nullptr;
      }
      const int np = prec == NR_GEMM_BF16 ? 1 : 3;
      const int rc = BN == 256 ? (np == 1 ? launch_big_1_256(gb, am, bmode, sp, stream) : launch_big_3_256(gb, am, bmode, sp, stream))
                               : (np == 1 ? launch_big_1_128(gb, am, bmode, sp, stream) : launch_big_3_128(gb, am, bmode, sp, stream));
      if (rc == NR_OK && tail_ws) {
        hipLaunchKernelGGL(tail_reduce_kernel, dim3(1024), dim3(256), 0, stream, C, ldc, work, g.Cm.idx, g.pad_row,
                           M, m_dev, N, g.vec);
        NR_LAUNCH_CHECK();
      }
      if (rc == NR_OK && slab) {
        int64_t blocks = (M * ((N + 3) / 4) + 255) / 256;
        blocks = blocks > 2048 ? 2048 : (blocks < 1 ? 1 : blocks);
        hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, C, ldc, work, sld,
                           gb.slab_stride, sp, M, N, K, gb.kchunk, m_dev, k_dev, g.vec, gb.colsum);
        NR_LAUNCH_CHECK();
        if (fold && colsum_folded) *colsum_folded = 1;
      }
      if (rc != -1) return rc;
    }
  }
  if (bm == 128 && bn == 128) return launch_modes<128, 128>(g, am, bmode, splits, prec, stream);
  if (bm == 64 && bn == 64) return launch_modes64(g, am, bmode, splits, stream);
  return -1;
}
