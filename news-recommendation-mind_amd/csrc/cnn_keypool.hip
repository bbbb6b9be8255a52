// Fused word-attention head of the CNN news encoder (models/Encoders/CNN.py:18-24,44-46 over the
// conv output C of CNN.py:41-42), one workgroup per title of L <= 32 tokens:
//
//   K   = tanh(C Wqᵀ + bq)                     wordQueryProject + Tanh (CNN.py:46)
//   s_l = q · K_l / sqrt(H),  p = XSoftmax(s, mask),  news = Σ_l p_l C_l
//                                              scaled_dp_attention (Attention.py:5-30)
//
// and its whole backward in ONE pass over C per title: the key projection is read back from the
// forward's optional K output (kout / kin) or recomputed, dp_l = dnews · C_l, ds = p (dp - Σ p dp) / sqrt(H), dK = ds q (1 - K²),
// dC = p dnews + dK Wq (+ dz) gated by ReLU'(C) (the conv pre-activation gradient), and the
// parameter gradients dWq = Σ dKᵀ C, dbq = Σ dK, dq = Σ ds K, dconv_b = Σ gated dC accumulate in
// registers / LDS across the titles of a persistent workgroup; each workgroup stores one partial and
// two reduce kernels add the partials in a fixed order (deterministic, no atomics).
// This replaces the T x Hp key GEMM + tanh epilogue, the word pooling, its backward, the key
// dgrad / wgrad GEMMs and two bias column sums: seven launches and four T x Hp round trips.
//
// Layout: Hp = 32 NB <= 160 (the conv width padded; the backward's per-wave dWq accumulators, 16 NB
// registers, spill past NB = 5, C / Wq / bq / q exactly zero past H); wave w of the
// NB waves owns output column block w of K, of dC and of dWq's rows.  Products on the matrix
// cores in the caller's GEMM arithmetic (mfma_planes.h: 0 = f32 MFMA, 3 = bf16x6, 1 = bf16), each
// 32 x 32 output block over 16-value per-lane fragments, lane (c, h) holding k = 32 chunk + 16 h +
// 0..15 (the same k order in both operands).  Operand sources: C and dK tiles from LDS (row reads
// as ds_read_b128, column reads as ds_read_b32 -- both conflict-free at a row stride of Hp + 4
// floats); Wq rows / columns straight from L2 (100 KB at H = 150, shared by every workgroup).
#include "common.h"
#include "../../include/newsrec_hip.h"
#include "mfma_planes.h"

namespace {

struct KPArgs {
  const float* c; int64_t ldc;        // [T][Hp] conv output after ReLU (zero past H)
  const float* wq;                    // [Hp][Hp] padded key projection (row j = output, col k = input)
  const float* bq;                    // [Hp]
  const float* q; int qn;             // query [qn] (qn = H), zero past qn
  const void* mask; int mask_dt;      // [nseq][L] (forward)
  int64_t nseq; int L; float scale;
  float* news; int64_t ldn;           // fwd: [nseq][Hp]
  float* probs;                       // fwd out / bwd in: [T]
  const float* dnews; int64_t lddn;   // bwd: [nseq][>= qn]
  const float* dz; int64_t lddz;      // bwd (optional): gradient of the token output C, [T][>= H]
  int H;
  float* dc; int64_t lddc;            // bwd out: [T][Hp] gated dC (zero past H)
  float* ws;                          // bwd: [gridDim.x][nws] partials: dwq | dbq | dq | dconv_b
  int64_t nws;
  float* kout; int64_t ldk;           // fwd (optional): K = tanh(C Wqᵀ + bq), [T][Hp]
  const float* kin;                   // bwd (optional): the forward's K (skips the key recompute)
};

// 16-B aligned: without it hipcc cannot prove the float4 row reads / writes aligned and splits each
// into ds_read2_b32 / ds_write2_b32, whose 32-bank addressing puts the 32 rows of one column (row
// stride Hp + 4 = 164 dwords, 4 mod 32) on 8 banks: the 7.45 (fwd) / 3.49 (bwd) extra LDS cycles per
// instruction of the round-3 PMC (profiles/r03_l_pmc_keypool_*.json)
template <int NB>
struct alignas(16) KPShared {
  static constexpr int HP = 32 * NB, SW = HP + 4;
  float ct[32][SW];   // C tile (rows >= L zero)
  float dk[32][SW];   // bwd: dK tile; fwd: K_j q_j products
  float p[32];
  float dpp[NB][32];   // bwd: column wave w's partial dp over its 32 columns
  float dsw[NB][32];   // bwd: ds as column wave w formed it (wave-private)
  float dn[HP], qv[HP], bq[HP];
};

// acc = C Wqᵀ for output columns 32 w .. 32 w + 31 (rows = the title's 32 token slots); B (Wq rows)
// from L2, one chunk ahead of its MFMAs.
template <int NB>
__device__ __forceinline__ void load_wrow(const KPArgs& g, int w, int c, int h, int ch, float (&b)[16]) {
  constexpr int HP = 32 * NB;
  const float* wrow = g.wq + (int64_t)(32 * w + c) * HP + 16 * h + 32 * ch;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const float4 y = *reinterpret_cast<const float4*>(wrow + 4 * u);
    b[4 * u] = y.x; b[4 * u + 1] = y.y; b[4 * u + 2] = y.z; b[4 * u + 3] = y.w;
  }
}

template <int NB>
__device__ __forceinline__ void load_crow(const KPShared<NB>& sm, int c, int h, int ch, float (&a)[16]) {
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const float4 x = *reinterpret_cast<const float4*>(&sm.ct[c][32 * ch + 16 * h + 4 * u]);
    a[4 * u] = x.x; a[4 * u + 1] = x.y; a[4 * u + 2] = x.z; a[4 * u + 3] = x.w;
  }
}

template <int NB, int NP>
__device__ __forceinline__ void key_block(const KPArgs& g, const KPShared<NB>& sm, int w, int c, int h, f32x16& acc) {
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  float bn[16];
  load_wrow<NB>(g, w, c, h, 0, bn);
#pragma unroll 1
  for (int ch = 0; ch < NB; ++ch) {   // one chunk's fragments live at a time, the next one's B in flight
    float a[16], b[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) b[s] = bn[s];
    if (ch + 1 < NB) load_wrow<NB>(g, w, c, h, ch + 1, bn);
    load_crow<NB>(sm, c, h, ch, a);
    mfma16<NP>(acc, a, b);
  }
}

template <int NB>
__device__ __forceinline__ void stage_vectors(const KPArgs& g, KPShared<NB>& sm) {
  constexpr int HP = 32 * NB;
  for (int k = threadIdx.x; k < HP; k += 64 * NB) {
    sm.qv[k] = k < g.qn ? g.q[k] : 0.f;
    sm.bq[k] = g.bq[k];
  }
}

template <int NB, int NP>
__global__ __launch_bounds__(64 * NB) void cnn_keypool_fwd_kernel(KPArgs g) {
  constexpr int HP = 32 * NB;
  __shared__ KPShared<NB> sm;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, c = lane & 31, h = lane >> 5;
  stage_vectors<NB>(g, sm);
  constexpr int Q4 = 8 * NB;
  constexpr int TPF = (32 * Q4 + 64 * NB - 1) / (64 * NB);   // C-tile float4 per thread
  float4 cn[TPF];   // the next title's C tile travels in registers while this one computes
  auto fetch = [&](int64_t seq) {
#pragma unroll
    for (int u = 0; u < TPF; ++u) {
      const int i = tid + u * 64 * NB;
      const int r = i / Q4, c4 = i - r * Q4;
      const bool ok = i < 32 * Q4 && r < g.L;
      cn[u] = *reinterpret_cast<const float4*>(g.c + (seq * g.L + (ok ? r : 0)) * g.ldc + 4 * (ok ? c4 : 0));
      if (!ok) cn[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  if ((int64_t)blockIdx.x < g.nseq) fetch(blockIdx.x);
  for (int64_t seq = blockIdx.x; seq < g.nseq; seq += gridDim.x) {
    __syncthreads();   // the previous title's pooling reads of ct are done
#pragma unroll
    for (int u = 0; u < TPF; ++u) {
      const int i = tid + u * 64 * NB;
      if (i < 32 * Q4) *reinterpret_cast<float4*>(&sm.ct[i / Q4][4 * (i % Q4)]) = cn[u];
    }
    __syncthreads();
    if (seq + gridDim.x < g.nseq) fetch(seq + gridDim.x);
    {
      f32x16 acc;
      key_block<NB, NP>(g, sm, w, c, h, acc);
      const int j = 32 * w + c;
      const float bj = sm.bq[j];
#pragma unroll
      for (int r = 0; r < 16; ++r) sm.dk[crow(r, h)][j] = tanhf(acc[r] + bj);
    }
    __syncthreads();
    if (g.kout) {   // K rows < L to HBM as float4 rows from LDS (per-lane column stores from the
                    // MFMA layout kept 16 64-bit addresses live: 159 VGPRs, two workgroups per CU)
      for (int i = tid; i < g.L * Q4; i += 64 * NB) {
        const int r = i / Q4, c4 = i - r * Q4;
        *reinterpret_cast<float4*>(g.kout + (seq * g.L + r) * g.ldk + 4 * c4) =
            *reinterpret_cast<const float4*>(&sm.dk[r][4 * c4]);
      }
    }
    if (w == 0) {   // scores and the masked softmax, lane l = token l
      const int l = lane & 31;
      float s = 0.f;
#pragma unroll 4
      for (int k4 = 0; k4 < HP / 4; ++k4) {
        const float4 v = *reinterpret_cast<const float4*>(&sm.dk[l][4 * k4]);
        const float4 qv = *reinterpret_cast<const float4*>(&sm.qv[4 * k4]);
        s += (v.x * qv.x + v.y * qv.y) + (v.z * qv.z + v.w * qv.w);
      }
      const bool keep = lane < g.L && nr_mask_at(g.mask, g.mask_dt, seq * g.L + lane);
      const float v = keep ? s * g.scale : -INFINITY;
      const float mx = nr_wave_max(v);
      const float e = keep ? __expf(v - mx) : 0.f;
      const float sum = nr_wave_sum(e);
      const float p = sum > 0.f ? e / sum : 0.f;
      if (lane < 32) sm.p[lane] = p;
      if (lane < g.L) g.probs[seq * g.L + lane] = p;
    }
    __syncthreads();
    for (int k = tid; k < HP; k += 64 * NB) {   // news = Σ_l p_l C_l
      float acc = 0.f;
      for (int l = 0; l < g.L; ++l) acc = fmaf(sm.p[l], sm.ct[l][k], acc);
      g.news[seq * g.ldn + k] = acc;
    }
  }
}

// buffer resource word 3 (gfx9 family: 32-bit data format, raw addressing)
constexpr int kBufWord3 = 0x00020000;

// Forward on the bf16 MFMA (NP = 3: bf16x6, NP = 1: bf16) with the C tile split ONCE: the staging
// threads write each C element's bf16 planes to LDS (the f32 form's key products had every column
// wave split all of C again, NB times per title: ~1.4 K VALU per wave and title, half the kernel's
// issue), the key products read the A fragments as ds_read_b128 of the planes, the scores are
// reduced across the wave's 32 columns in registers (no K tile in LDS; the optional K output goes
// out through buffer stores) and the pooling reads C back
// as h + m + l (exact: the split's residuals are exact and the last is 8 bits wide) or, for
// bf16, from the f32 tile kept beside its one plane.
__device__ __forceinline__ float bf16f(uint16_t v) { return __uint_as_float((uint32_t)v << 16); }

template <int NB, int NP>
struct alignas(16) KPPShared {
  static constexpr int HP = 32 * NB, SWB = HP + 8, SW = HP + 4;   // 84 dwords per plane row: ds_read_b128 conflict-free
  uint16_t cp[NP][32][SWB];                 // C tile planes (rows >= L zero)
  float ct[NP == 1 ? 32 : 1][SW];           // bf16: the f32 C tile for the pooling
  float ps[NB][32];                         // per column-wave partial scores
  float p[32];
  float qv[HP], bq[HP];
};

template <int NB, int NP>
__global__ __launch_bounds__(64 * NB) void cnn_keypool_fwd_planes_kernel(KPArgs g) {
  constexpr int HP = 32 * NB;
  using SM = KPPShared<NB, NP>;
  __shared__ SM sm;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, c = lane & 31, h = lane >> 5;
  for (int k = tid; k < HP; k += 64 * NB) {
    sm.qv[k] = k < g.qn ? g.q[k] : 0.f;
    sm.bq[k] = g.bq[k];
  }
  constexpr int Q4 = 8 * NB;
  constexpr int TPF = (32 * Q4 + 64 * NB - 1) / (64 * NB);   // C-tile float4 per thread
  float4 cn[TPF];   // the next title's C tile travels in registers while this one computes
  auto fetch = [&](int64_t seq) {
#pragma unroll
    for (int u = 0; u < TPF; ++u) {
      const int i = tid + u * 64 * NB;
      const int r = i / Q4, c4 = i - r * Q4;
      const bool ok = i < 32 * Q4 && r < g.L;
      cn[u] = *reinterpret_cast<const float4*>(g.c + (seq * g.L + (ok ? r : 0)) * g.ldc + 4 * (ok ? c4 : 0));
      if (!ok) cn[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  const int j = 32 * w + c;   // this lane's output column of K
  if ((int64_t)blockIdx.x < g.nseq) fetch(blockIdx.x);
  for (int64_t seq = blockIdx.x; seq < g.nseq; seq += gridDim.x) {
    __syncthreads();   // the previous title's reads of cp / ct / p are done
#pragma unroll
    for (int u = 0; u < TPF; ++u) {
      const int i = tid + u * 64 * NB;
      if (i < 32 * Q4) {
        const int r = i / Q4, k = 4 * (i % Q4);
        const float4 x = cn[u];
        if constexpr (NP == 1) {
          *reinterpret_cast<uint2*>(&sm.cp[0][r][k]) = nrfast::hi4(x.x, x.y, x.z, x.w);
          *reinterpret_cast<float4*>(&sm.ct[r][k]) = x;
        } else {
          uint2 p0, p1, p2;
          nrfast::split4(x.x, x.y, x.z, x.w, p0, p1, p2);
          *reinterpret_cast<uint2*>(&sm.cp[0][r][k]) = p0;
          *reinterpret_cast<uint2*>(&sm.cp[1][r][k]) = p1;
          *reinterpret_cast<uint2*>(&sm.cp[2][r][k]) = p2;
        }
      }
    }
    __syncthreads();
    if (seq + gridDim.x < g.nseq) fetch(seq + gridDim.x);
    {
      // acc = C Wqᵀ for output columns 32 w .. 32 w + 31; k order: lane (c, h) step m of chunk ch
      // holds k = 32 ch + 16 h + 8 m + 0..7 in both operands (A from the planes, B = Wq row j from L2)
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
      float bn[16];
      load_wrow<NB>(g, w, c, h, 0, bn);
#pragma unroll 1
      for (int ch = 0; ch < NB; ++ch) {
        float b[16];
#pragma unroll
        for (int s2 = 0; s2 < 16; ++s2) b[s2] = bn[s2];
        if (ch + 1 < NB) load_wrow<NB>(g, w, c, h, ch + 1, bn);
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          Planes<NP> a;
#pragma unroll
          for (int pl = 0; pl < NP; ++pl)
            a.v[pl] = *reinterpret_cast<const bf16x8*>(&sm.cp[pl][c][32 * ch + 16 * h + 8 * m]);
          mfma_x<NP>(acc, a, planes8<NP>(b + 8 * m));
        }
      }
      // s_l partial over this wave's 32 columns: tanh(acc + bq_j) q_j summed across the 32 lanes of
      // each half (rows crow(r, h))
      // (a butterfly: at lane distance 16, 8, 4, 2 each lane keeps the half of its registers its bit
      // selects and adds the partner's copy of it -- 8 + 4 + 2 + 1 exchanges instead of 16 x 5 -- then
      // one more at distance 1; lane c then holds row register r = (c >> 1) & 15's full sum)
      const float bj = sm.bq[j], qj = sm.qv[j];
      float kv[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) kv[r] = tanhf(acc[r] + bj);
      if (g.kout) {
        // K to HBM through a buffer resource over this title's L rows: one lane offset (row 4 h,
        // column j) plus a uniform per-register row offset, rows >= L dropped by the range check
        // (per-lane 64-bit addresses for the 16 stores took the kernel to 159 VGPRs: two workgroups
        // per CU instead of three)
        const __amdgpu_buffer_rsrc_t kr = __builtin_amdgcn_make_buffer_rsrc(
            g.kout + seq * g.L * g.ldk, (short)0, (int)(g.L * g.ldk * 4), kBufWord3);
        const int vo = (int)((4 * h * g.ldk + j) * 4);
#pragma unroll
        for (int r = 0; r < 16; ++r)
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(kv[r]), kr, vo,
                                                (int)(((r & 3) + 8 * (r >> 2)) * g.ldk * 4), 0);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) kv[r] *= qj;
#pragma unroll
      for (int st = 0; st < 4; ++st) {
        const int half = 8 >> st, d = 16 >> st;
        const bool up = (c & d) != 0;
#pragma unroll
        for (int i = 0; i < half; ++i) {
          const float keep = up ? kv[i + half] : kv[i], give = up ? kv[i] : kv[i + half];
          kv[i] = keep + __shfl_xor(give, d, 64);
        }
      }
      const float tot = kv[0] + __shfl_xor(kv[0], 1, 64);
      if ((c & 1) == 0) sm.ps[w][crow((c >> 1) & 15, h)] = tot;
    }
    __syncthreads();
    if (w == 0) {   // scores and the masked softmax, lane l = token l
      const int l = lane & 31;
      float s = 0.f;
#pragma unroll
      for (int ww = 0; ww < NB; ++ww) s += sm.ps[ww][l];
      const bool keep = lane < g.L && nr_mask_at(g.mask, g.mask_dt, seq * g.L + lane);
      const float v = keep ? s * g.scale : -INFINITY;
      const float mx = nr_wave_max(v);
      const float e = keep ? __expf(v - mx) : 0.f;
      const float sum = nr_wave_sum(e);
      const float pr = sum > 0.f ? e / sum : 0.f;
      if (lane < 32) sm.p[lane] = pr;
      if (lane < g.L) g.probs[seq * g.L + lane] = pr;
    }
    __syncthreads();
    for (int k = tid; k < HP; k += 64 * NB) {   // news = Σ_l p_l C_l
      float a = 0.f;
      for (int l = 0; l < g.L; ++l) {
        float x;
        if constexpr (NP == 1) {
          x = sm.ct[l][k];
        } else {
          x = (bf16f(sm.cp[0][l][k]) + bf16f(sm.cp[1][l][k])) + bf16f(sm.cp[2][l][k]);
        }
        a = fmaf(sm.p[l], x, a);
      }
      g.news[seq * g.ldn + k] = a;
    }
  }
}

// Backward: KP_BW = 8 waves (one workgroup per CU, two waves per SIMD).  Waves 0 .. NB-1 are COLUMN
// waves (key block, dK block and dC block w); the other 8 - NB are dWq waves, each owning a fixed
// share of dWq's NB² 32 x 32 blocks (bf16x6: a kb-major range; otherwise round-robin), accumulated
// across the workgroup's titles in LDS ([block][register][lane]: conflict-free, 100 KB at NB = 5 -- in registers they would cost every
// wave 144 VGPRs and spill) and computed while the column waves run the dC products; the column
// waves also form dp (each over its own 32 columns) and ds.  With NB = 5 each SIMD carries 18-20
// fragment products per title (five column waves on four SIMDs alone would leave one SIMD with
// twice the others' work).
constexpr int KP_BW = 8;

template <int NB>
constexpr int kp_maxb() { return (NB * NB + (KP_BW - NB) - 1) / (KP_BW - NB); }

// SK: the forward's K is read (g.kin, prefetched with the next title's C tile) instead of recomputed:
// the key products and their Wq row loads leave the kernel
template <int NB, int NP, bool SK>
__global__ __launch_bounds__(64 * KP_BW) void cnn_keypool_bwd_kernel(KPArgs g) {
  static_assert(NB >= 1 && NB < KP_BW, "column waves + at least one dWq wave");
  constexpr int HP = 32 * NB;
  constexpr int ND = KP_BW - NB;        // dWq waves
  constexpr int MAXB = kp_maxb<NB>();   // dWq blocks per dWq wave
  constexpr int Q4 = 8 * NB;            // float4 per C row
  constexpr int TPF = (32 * Q4 + 64 * KP_BW - 1) / (64 * KP_BW);   // C-tile float4 per thread
  __shared__ KPShared<NB> sm;
  __shared__ __attribute__((aligned(16))) float wacc[NB * NB][16][64];   // dWq block b: rows 32 jb + crow(r, h), columns 32 kb + c
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, c = lane & 31, h = lane >> 5;
  const bool colw = w < NB;
  const int d = w - NB;                 // dWq wave index (when !colw)
  for (int k = tid; k < HP; k += 64 * KP_BW) {
    sm.qv[k] = k < g.qn ? g.q[k] : 0.f;
    sm.bq[k] = g.bq[k];
  }
  for (int i = tid; i < NB * NB * 16 * 64; i += 64 * KP_BW) (&wacc[0][0][0])[i] = 0.f;
  float dq_acc = 0.f, dbq_acc = 0.f, dcb_acc = 0.f;
  const int j = 32 * (colw ? w : 0) + c;   // a column wave lane's column of K / dK / dC
  // a column wave's Wq column fragments (the dC products: 32 w + c, every chunk) for every title; the
  // row fragments of the key products come from L2 one chunk ahead (both sets would spill)
  constexpr bool WC_REGS = NP != 3;   // bf16x6: the operand split needs those registers (51 VGPRs spilled even without the key products)
  float wc[WC_REGS ? NB : 1][16];
  if (WC_REGS && colw) {
#pragma unroll
    for (int ch = 0; ch < NB; ++ch)
#pragma unroll
      for (int s2 = 0; s2 < 16; ++s2) wc[ch][s2] = g.wq[(int64_t)(32 * ch + 16 * h + s2) * HP + j];
  }
  // the next title's C tile / probabilities / dnews travel in registers while this one computes
  float4 cn[TPF];
  float pn = 0.f, dnn = 0.f;
  float kn[16];   // with the forward's K: a column wave lane's 16 K values of the next title
  auto fetch = [&](int64_t seq) {
    if (SK && colw) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int tok = crow(r, h);
        kn[r] = tok < g.L ? g.kin[(seq * g.L + tok) * g.ldk + j] : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < TPF; ++u) {
      const int i = tid + u * 64 * KP_BW;
      const int r = i / Q4, c4 = i - r * Q4;
      const bool ok = i < 32 * Q4 && r < g.L;
      cn[u] = *reinterpret_cast<const float4*>(g.c + (seq * g.L + (ok ? r : 0)) * g.ldc + 4 * (ok ? c4 : 0));
      if (!ok) cn[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (tid < 32) pn = tid < g.L ? g.probs[seq * g.L + tid] : 0.f;
    if (tid >= 64 && tid < 64 + HP) dnn = tid - 64 < g.qn ? g.dnews[seq * g.lddn + tid - 64] : 0.f;
  };
  if ((int64_t)blockIdx.x < g.nseq) fetch(blockIdx.x);
  for (int64_t seq = blockIdx.x; seq < g.nseq; seq += gridDim.x) {
    __syncthreads();   // the previous title's reads of ct / dk / p / dn are done
#pragma unroll
    for (int u = 0; u < TPF; ++u) {
      const int i = tid + u * 64 * KP_BW;
      if (i < 32 * Q4) *reinterpret_cast<float4*>(&sm.ct[i / Q4][4 * (i % Q4)]) = cn[u];
    }
    if (tid < 32) sm.p[tid] = pn;
    if (tid >= 64 && tid < 64 + HP) sm.dn[tid - 64] = dnn;
    float kr[16];
    if (SK && colw) {   // (before the next title's fetch reuses kn)
#pragma unroll
      for (int r = 0; r < 16; ++r) kr[r] = kn[r];
    }
    __syncthreads();
    if (seq + gridDim.x < g.nseq) fetch(seq + gridDim.x);
    if (!SK && colw) {
      f32x16 acc;
      key_block<NB, NP>(g, sm, w, c, h, acc);
      const float bj = sm.bq[j];
#pragma unroll
      for (int r = 0; r < 16; ++r) kr[r] = tanhf(acc[r] + bj);
    }
    if (colw) {   // dp_l = dnews · C_l, this wave's 32 columns: lane (c, h) = token c, columns 32 w + 16 h + 0..15
      float dp = 0.f;
#pragma unroll 1
      for (int u = 0; u < 4; ++u) {
        const float4 x = *reinterpret_cast<const float4*>(&sm.ct[c][32 * w + 16 * h + 4 * u]);
        const float4 dv = *reinterpret_cast<const float4*>(&sm.dn[32 * w + 16 * h + 4 * u]);
        dp = fmaf(x.x, dv.x, dp); dp = fmaf(x.y, dv.y, dp);
        dp = fmaf(x.z, dv.z, dp); dp = fmaf(x.w, dv.w, dp);
      }
      dp += __shfl_xor(dp, 32, 64);
      if (h == 0) sm.dpp[w][c] = dp;
    }
    __syncthreads();
    if (colw) {
      // ds = p (dp - Σ p dp) scale, formed by every column wave from the same partials in the same
      // order (identical values) into its own LDS row: no workgroup barrier before the reads
      float dp = 0.f;
#pragma unroll
      for (int ww = 0; ww < NB; ++ww) dp += sm.dpp[ww][c];
      const float pl = sm.p[c];
      const float rs = nr_wave_sum(h == 0 ? pl * dp : 0.f);
      if (h == 0) sm.dsw[w][c] = pl * (dp - rs) * g.scale;
      wave_lds_fence();
      const float qj = sm.qv[j];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int tok = crow(r, h);
        const float dsr = sm.dsw[w][tok];
        dq_acc = fmaf(dsr, kr[r], dq_acc);
        const float dkv = dsr * qj * (1.f - kr[r] * kr[r]);
        dbq_acc += dkv;
        sm.dk[tok][j] = dkv;
      }
    }
    __syncthreads();
    if (colw) {   // dC block w = dK Wq (+ p dnews + dz), gated by ReLU'(C)
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
      if constexpr (WC_REGS) {
#pragma unroll
        for (int ch = 0; ch < NB; ++ch) {
          float a[16];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const float4 x = *reinterpret_cast<const float4*>(&sm.dk[c][32 * ch + 16 * h + 4 * u]);
            a[4 * u] = x.x; a[4 * u + 1] = x.y; a[4 * u + 2] = x.z; a[4 * u + 3] = x.w;
          }
          mfma16<NP>(acc, a, wc[ch]);
        }
      } else {
        const float* wcol = g.wq + (int64_t)(16 * h) * HP + j;
        float bn[16];
#pragma unroll
        for (int s2 = 0; s2 < 16; ++s2) bn[s2] = wcol[(int64_t)s2 * HP];
#pragma unroll 1
        for (int ch = 0; ch < NB; ++ch) {   // the next chunk's Wq column fragment in flight
          float a[16], b[16];
#pragma unroll
          for (int s2 = 0; s2 < 16; ++s2) b[s2] = bn[s2];
          if (ch + 1 < NB) {
#pragma unroll
            for (int s2 = 0; s2 < 16; ++s2) bn[s2] = wcol[(int64_t)(32 * (ch + 1) + s2) * HP];
          }
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const float4 x = *reinterpret_cast<const float4*>(&sm.dk[c][32 * ch + 16 * h + 4 * u]);
            a[4 * u] = x.x; a[4 * u + 1] = x.y; a[4 * u + 2] = x.z; a[4 * u + 3] = x.w;
          }
          mfma16<NP>(acc, a, b);
        }
      }
      const float dnj = sm.dn[j];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int tok = crow(r, h);
        float v = fmaf(sm.p[tok], dnj, acc[r]);
        if (tok < g.L) {
          if (g.dz && j < g.H) v += g.dz[(seq * g.L + tok) * g.lddz + j];
          const float gated = sm.ct[tok][j] > 0.f ? v : 0.f;
          g.dc[(seq * g.L + tok) * g.lddc + j] = gated;
          dcb_acc += gated;
        }
      }
    } else if constexpr (NP == 3) {   // dWq blocks of this wave += dKᵀ C over the title's tokens
      // bf16x6: a contiguous kb-major range of blocks, C column block kb (the B operand) read and
      // split once per kb and reused across the range's jb (round-robin blocks split both operands
      // of every block: 18 splits per title on the busiest wave at NB = 5, now 11; backward 94.0 ->
      // 90.5 us, profiles/r04_m_*).  bf16's split is one rounding: the round-robin form below
      // measured faster there (53.4 vs 58.0 us).
      const int b0 = d * NB * NB / ND, b1 = (d + 1) * NB * NB / ND;
      float bb[16];
      Planes<NP> bp[2];
#pragma unroll 1
      for (int i = 0; i < MAXB; ++i) {
        const int bq = b0 + i;
        if (bq < b1) {
          const int kb = bq / NB, jb = bq - kb * NB;
          if (i == 0 || jb == 0) {
#pragma unroll
            for (int s2 = 0; s2 < 16; ++s2) bb[s2] = sm.ct[16 * h + s2][32 * kb + c];
            bp[0] = planes8<NP>(bb);
            bp[1] = planes8<NP>(bb + 8);
          }
          float a[16];
#pragma unroll
          for (int s2 = 0; s2 < 16; ++s2) a[s2] = sm.dk[16 * h + s2][32 * jb + c];
          const int b = jb * NB + kb;   // accumulator slot (rows 32 jb.., columns 32 kb..)
          f32x16 acc;
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[r] = wacc[b][r][lane];
          mfma_x<NP>(acc, planes8<NP>(a), bp[0]);
          mfma_x<NP>(acc, planes8<NP>(a + 8), bp[1]);
#pragma unroll
          for (int r = 0; r < 16; ++r) wacc[b][r][lane] = acc[r];
        }
        __builtin_amdgcn_sched_barrier(0);   // keep the next block's fragment reads out of this one
      }
    } else {   // f32 / bf16: round-robin blocks, both fragments per block
#pragma unroll
      for (int i = 0; i < MAXB; ++i) {
        const int b = d + i * ND;
        if (b < NB * NB) {
          const int jb = b / NB, kb = b - jb * NB;
          float a[16], bb[16];
#pragma unroll
          for (int s2 = 0; s2 < 16; ++s2) {
            a[s2] = sm.dk[16 * h + s2][32 * jb + c];
            bb[s2] = sm.ct[16 * h + s2][32 * kb + c];
          }
          f32x16 acc;
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[r] = wacc[b][r][lane];
          mfma16<NP>(acc, a, bb);
#pragma unroll
          for (int r = 0; r < 16; ++r) wacc[b][r][lane] = acc[r];
        }
        __builtin_amdgcn_sched_barrier(0);   // keep the next block's fragment reads out of this one
      }
    }
  }
  // this workgroup's partials (every slot written, also by a workgroup without titles)
  __syncthreads();
  float* wsb = g.ws + (int64_t)blockIdx.x * g.nws;
  if (colw) {
    dq_acc += __shfl_xor(dq_acc, 32, 64);
    dbq_acc += __shfl_xor(dbq_acc, 32, 64);
    dcb_acc += __shfl_xor(dcb_acc, 32, 64);
    if (h == 0) {
      wsb[(int64_t)HP * HP + j] = dbq_acc;
      wsb[(int64_t)HP * HP + HP + j] = dq_acc;
      wsb[(int64_t)HP * HP + 2 * HP + j] = dcb_acc;
    }
  }
  for (int i = tid; i < NB * NB * 16 * 64; i += 64 * KP_BW) {   // dWq blocks, coalesced along columns
    const int b = i / (16 * 64), r = (i / 64) % 16, ln = i % 64;
    const int jb = b / NB, kb = b - jb * NB;
    wsb[(int64_t)(32 * jb + crow(r, ln >> 5)) * HP + 32 * kb + (ln & 31)] = wacc[b][r][ln];
  }
}

// Partials -> outputs in two deterministic stages: stage 1 sums slice y of the G workgroup
// partials (G / KP_SLICES each, eight loads in flight per thread) into part[y]; stage 2 adds the
// KP_SLICES slices in order and scatters to dwq [Hp][Hp], dbq [Hp], dq [qn], dconv_b [H] (stored).
// One pass over all G partials with one thread per column left the reads latency-bound.
constexpr int KP_SLICES = 8;

__global__ __launch_bounds__(256) void cnn_keypool_reduce1_kernel(const float* __restrict__ ws, int64_t nws, int G,
                                                                  float* __restrict__ part) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= nws) return;
  const int y = blockIdx.y;
  const int g0 = (int)((int64_t)G * y / KP_SLICES), g1 = (int)((int64_t)G * (y + 1) / KP_SLICES);
  float s = 0.f;
  int g = g0;
  for (; g + 8 <= g1; g += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = ws[(int64_t)(g + u) * nws + i];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  for (; g < g1; ++g) s += ws[(int64_t)g * nws + i];
  part[(int64_t)y * nws + i] = s;
}

__global__ __launch_bounds__(256) void cnn_keypool_reduce2_kernel(const float* __restrict__ part, int64_t nws,
                                                                  int HP, int qn, int H, float* __restrict__ dwq,
                                                                  float* __restrict__ dbq, float* __restrict__ dq,
                                                                  float* __restrict__ dcb) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= nws) return;
  float v[KP_SLICES];
#pragma unroll
  for (int y = 0; y < KP_SLICES; ++y) v[y] = part[(int64_t)y * nws + i];
  float s = 0.f;
#pragma unroll
  for (int y = 0; y < KP_SLICES; ++y) s += v[y];
  const int64_t hh = (int64_t)HP * HP;
  if (i < hh) {
    dwq[i] = s;
  } else if (i < hh + HP) {
    dbq[i - hh] = s;
  } else if (i < hh + 2 * HP) {
    if (i - hh - HP < qn) dq[i - hh - HP] = s;
  } else if (i - hh - 2 * HP < H) {
    dcb[i - hh - 2 * HP] = s;
  }
}

int g_cus = 0;
int cu_count() {
  if (g_cus == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess)
      g_cus = n;
    if (g_cus <= 0) g_cus = 256;
  }
  return g_cus;
}

// persistent workgroups per CU: the forward (NB waves, 44 KB of LDS, <= 128 VGPRs) three, the backward (8 waves,
// 147 KB of LDS) one
int64_t kp_groups(int64_t nseq, int per_cu) {
  const int64_t cap = (int64_t)cu_count() * per_cu;
  return nseq < cap ? (nseq > 0 ? nseq : 1) : cap;
}

bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// A persistent grid larger than what is resident leaves a tail of workgroups that start only when
// others finish: the forward's grid is capped by the instantiation's occupancy (at 159 VGPRs the
// bf16x6 forward fitted two workgroups per CU, not three, and ran 52 -> 76 us)
template <typename Kern>
int resident_per_cu(Kern kern, int nt, int want) {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kern, nt, 0) != hipSuccess || n < 1) n = 1;
  return n < want ? n : want;
}

// f32 MFMA: the per-wave fp32 fragments; bf16x6 / bf16: the C tile split once into LDS planes
template <int NB, int NP>
void launch_fwd(const KPArgs& g, hipStream_t s) {
  static int per_cu = 0;   // resident workgroups per CU of this instantiation, queried once
  if constexpr (NP == 0) {
    if (per_cu == 0) per_cu = resident_per_cu(cnn_keypool_fwd_kernel<NB, NP>, 64 * NB, 3);
    hipLaunchKernelGGL((cnn_keypool_fwd_kernel<NB, NP>), dim3((unsigned)kp_groups(g.nseq, per_cu)), dim3(64 * NB), 0, s, g);
  } else {
    if (per_cu == 0) per_cu = resident_per_cu(cnn_keypool_fwd_planes_kernel<NB, NP>, 64 * NB, 3);
    hipLaunchKernelGGL((cnn_keypool_fwd_planes_kernel<NB, NP>), dim3((unsigned)kp_groups(g.nseq, per_cu)), dim3(64 * NB),
                       0, s, g);
  }
}

template <int NB>
int launch_cnn_keypool_fwd_kernel(int np, const KPArgs& g, hipStream_t s) {
  if (np == 0) launch_fwd<NB, 0>(g, s);
  else if (np == 1) launch_fwd<NB, 1>(g, s);
  else launch_fwd<NB, 3>(g, s);
  NR_LAUNCH_CHECK();
  return NR_OK;
}
template <int NB>
int launch_cnn_keypool_bwd_kernel(int np, const KPArgs& g, int64_t grid, hipStream_t s) {
#define NR_KPB(NP_)                                                                                       \
  if (g.kin) hipLaunchKernelGGL((cnn_keypool_bwd_kernel<NB, NP_, true>), dim3((unsigned)grid), dim3(64 * KP_BW), 0, s, g); \
  else hipLaunchKernelGGL((cnn_keypool_bwd_kernel<NB, NP_, false>), dim3((unsigned)grid), dim3(64 * KP_BW), 0, s, g);
  if (np == 0) { NR_KPB(0) } else if (np == 1) { NR_KPB(1) } else { NR_KPB(3) }
#undef NR_KPB
  NR_LAUNCH_CHECK();
  return NR_OK;
}

int np_of(int prec) { return prec == NR_GEMM_F32 ? 0 : prec == NR_GEMM_BF16 ? 1 : 3; }

}  // namespace

extern "C" int64_t nr_cnn_keypool_workspace(int64_t nseq, int32_t Hp) {
  if (nseq < 0 || Hp < 32 || Hp > 160 || (Hp & 31)) return -1;
  return (kp_groups(nseq, 1) + KP_SLICES) * ((int64_t)Hp * Hp + 3 * (int64_t)Hp);
}

extern "C" int nr_cnn_keypool_fwd(const float* C, int64_t ldc, const float* wq, const float* bq, const float* q,
                                  int32_t qn, const void* mask, int32_t mask_dtype, int64_t nseq, int32_t L,
                                  int32_t Hp, float scale, int32_t prec, float* news, int64_t ldn, float* probs,
                                  float* kout, int64_t ldk, hipStream_t stream) {
  if (Hp < 32 || Hp > 160 || (Hp & 31) || L < 1 || L > 32 || qn < 1 || qn > Hp || nseq < 0 || ldc < Hp ||
      (ldc & 3) || ldn < Hp)
    return NR_EINVAL(0);
  if (!C || !wq || !bq || !q || !mask || !news || !probs) return NR_EINVAL(1);
  if (!al16(C) || !al16(wq)) return NR_EINVAL(2);
  // (the buffer-store K output addresses one title's L rows with a 32-bit byte range)
  if (kout && (ldk < Hp || (ldk & 3) || !al16(kout) || (int64_t)L * ldk * 4 > INT32_MAX)) return NR_EINVAL(3);
  if (nseq == 0) return NR_OK;
  KPArgs g{};
  g.c = C; g.ldc = ldc; g.wq = wq; g.bq = bq; g.q = q; g.qn = qn; g.mask = mask; g.mask_dt = mask_dtype;
  g.nseq = nseq; g.L = L; g.scale = scale; g.news = news; g.ldn = ldn; g.probs = probs; g.H = qn;
  g.kout = kout; g.ldk = ldk;
  const int np = np_of(prec);
  switch (Hp / 32) {
    case 1: return launch_cnn_keypool_fwd_kernel<1>(np, g, stream);
    case 2: return launch_cnn_keypool_fwd_kernel<2>(np, g, stream);
    case 3: return launch_cnn_keypool_fwd_kernel<3>(np, g, stream);
    case 4: return launch_cnn_keypool_fwd_kernel<4>(np, g, stream);
    default: return launch_cnn_keypool_fwd_kernel<5>(np, g, stream);
  }
}

extern "C" int nr_cnn_keypool_bwd(const float* C, int64_t ldc, const float* wq, const float* bq, const float* q,
                                  int32_t qn, int64_t nseq, int32_t L, int32_t Hp, int32_t H, float scale,
                                  int32_t prec, const float* probs, const float* dnews, int64_t lddn, const float* dz,
                                  int64_t lddz, float* dc, int64_t lddc, float* dwq, float* dbq, float* dq,
                                  float* dconv_b, float* ws, int64_t ws_floats, const float* kin, int64_t ldk,
                                  hipStream_t stream) {
  if (Hp < 32 || Hp > 160 || (Hp & 31) || L < 1 || L > 32 || qn < 1 || qn > Hp || H < 1 || H > Hp || nseq < 0 ||
      ldc < Hp || (ldc & 3) || lddn < qn || lddc < Hp || (dz && lddz < H))
    return NR_EINVAL(0);
  if (!C || !wq || !bq || !q || !probs || !dnews || !dc || !dwq || !dbq || !dq || !dconv_b || !ws) return NR_EINVAL(1);
  if (!al16(C) || !al16(wq)) return NR_EINVAL(2);
  if (kin && ldk < Hp) return NR_EINVAL(4);
  const int64_t nws = (int64_t)Hp * Hp + 3 * (int64_t)Hp;
  const int64_t grid = kp_groups(nseq, 1);
  if (ws_floats < (grid + KP_SLICES) * nws) return NR_EINVAL(3);
  KPArgs g{};
  g.c = C; g.ldc = ldc; g.wq = wq; g.bq = bq; g.q = q; g.qn = qn;
  g.nseq = nseq; g.L = L; g.scale = scale; g.probs = const_cast<float*>(probs);
  g.dnews = dnews; g.lddn = lddn; g.dz = dz; g.lddz = lddz; g.H = H; g.dc = dc; g.lddc = lddc;
  g.ws = ws; g.nws = nws;
  g.kin = kin; g.ldk = ldk;
  const int np = np_of(prec);
  int rc;
  switch (Hp / 32) {
    case 1: rc = launch_cnn_keypool_bwd_kernel<1>(np, g, grid, stream); break;
    case 2: rc = launch_cnn_keypool_bwd_kernel<2>(np, g, grid, stream); break;
    case 3: rc = launch_cnn_keypool_bwd_kernel<3>(np, g, grid, stream); break;
    case 4: rc = launch_cnn_keypool_bwd_kernel<4>(np, g, grid, stream); break;
    default: rc = launch_cnn_keypool_bwd_kernel<5>(np, g, grid, stream); break;
  }
  if (rc != NR_OK) return rc;
  float* part = ws + grid * nws;
  hipLaunchKernelGGL(cnn_keypool_reduce1_kernel, dim3((unsigned)((nws + 255) / 256), KP_SLICES), dim3(256), 0, stream,
                     ws, nws, (int)grid, part);
  NR_LAUNCH_CHECK();
  hipLaunchKernelGGL(cnn_keypool_reduce2_kernel, dim3((unsigned)((nws + 255) / 256)), dim3(256), 0, stream, part, nws,
                     Hp, qn, H, dwq, dbq, dq, dconv_b);
  NR_LAUNCH_CHECK();
  return NR_OK;
}
