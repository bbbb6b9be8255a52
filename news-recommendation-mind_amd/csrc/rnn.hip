// Recurrent user encoders over the click history (one layer, batch_first):
//   RNN_User_Encoder  (models/Encoders/RNN.py:50-73): LSTM or GRU, h0 = 0, run over
//                     pack_padded_sequence(lens = Σ his_mask), output h at step len-1
//   LSTUR_User_Encoder (models/Encoders/RNN.py:88-104): LSTM over the FLIPPED history, all N
//                     steps, h0 = userEmbedding[u] (gathered here), c0 = 0
// PyTorch gate layout: LSTM rows (i, f, g, o), GRU rows (r, z, n) of weight_ih / weight_hh.
//
// The input projections x_t W_ihᵀ + b_ih of all steps are one MFMA GEMM (nr_gemm_f32) before
// this kernel; here only the sequential part runs: one workgroup per sequence keeps h (and c)
// in LDS and, per step, computes h W_hhᵀ + b_hh with W_hh streamed from L2 in a transposed,
// coalesced layout.  The forward saves the activated gates and h_{t-1} (and c_{t-1}) of every
// step, so the backward is exact BPTT without recomputation, and the weight gradients become
// two more GEMMs: dW_ih = dGIᵀ X, dW_hh = dGHᵀ H_prev.
#include <stdlib.h>

#include "common.h"
#include "../../include/newsrec_hip.h"

namespace {

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }

struct RnnArgs {
  int cell;  // NR_CELL_LSTM / NR_CELL_GRU
  const float* gx; int64_t ldgx;
  const float* whh;           // fwd: W_hhᵀ [H][G*H];  bwd: W_hh [G*H][H]
  const float* bhh;
  const float* h0; int64_t ldh0; const int64_t* h0_idx;
  const void* mask; int mask_dt;
  int reverse;
  int64_t B; int N; int H;
  float* gates;               // [B*N][4H]
  float* hprev;               // [B*N][H]
  float* cprev;               // [B*N][H] (LSTM)
  float* hout; int64_t ldho;
  // bwd
  const float* dhout; int64_t lddho;
  float* dgi; float* dgh; int64_t lddg;
  float* dh0; int64_t lddh0;
};

__device__ int seq_len(const RnnArgs& g, int64_t b, int* red) {
  if (!g.mask) return g.N;
  int cnt = 0;
  for (int j = threadIdx.x; j < g.N; j += blockDim.x) cnt += nr_mask_at(g.mask, g.mask_dt, b * g.N + j) ? 1 : 0;
  atomicAdd(red, cnt);
  __syncthreads();
  const int len = *red;
  return len;
}

__global__ __launch_bounds__(256) void rnn_fwd_kernel(RnnArgs g) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int H = g.H, G = g.cell == NR_CELL_LSTM ? 4 : 3, GH = G * H;
  float* h = sm;            // [H]
  float* c = h + H;         // [H]
  float* gh = c + H;        // [GH]
  int* red = reinterpret_cast<int*>(gh + GH);
  const int64_t b = blockIdx.x;
  const int tid = threadIdx.x;
  if (tid == 0) *red = 0;
  for (int u = tid; u < H; u += blockDim.x) {
    float h0 = 0.f;
    if (g.h0) {
      const int64_t r = g.h0_idx ? g.h0_idx[b] : b;
      h0 = g.h0[r * g.ldh0 + u];
    }
    h[u] = h0;
    c[u] = 0.f;
  }
  __syncthreads();
  const int len = seq_len(g, b, red);
  // an all-zero mask row (len 0; pack_padded_sequence raises, MIND forces his_mask[0] = 1):
  // defined output h0, and the backward passes dh straight to dh0
  if (len == 0)
    for (int u = tid; u < H; u += blockDim.x) g.hout[b * g.ldho + u] = h[u];
  for (int t = 0; t < g.N; ++t) {
    const int tt = g.reverse ? g.N - 1 - t : t;
    const int64_t row = b * g.N + tt;
    if (t >= len) {   // padded steps: zero what the backward GEMMs read
      for (int r = tid; r < 4 * H; r += blockDim.x) g.gates[row * 4 * H + r] = 0.f;
      for (int u = tid; u < H; u += blockDim.x) {
        g.hprev[row * H + u] = 0.f;
        if (g.cprev) g.cprev[row * H + u] = 0.f;
      }
      continue;
    }
    for (int r = tid; r < GH; r += blockDim.x) {
      float acc = g.bhh ? g.bhh[r] : 0.f;
      const float* wc = g.whh + r;
      for (int k = 0; k < H; ++k) acc = fmaf(wc[(int64_t)k * GH], h[k], acc);
      gh[r] = acc;
    }
    __syncthreads();
    const float* xs = g.gx + row * g.ldgx;
    float hn[2], cn[2];
    int nu = 0;
    for (int u = tid; u < H; u += blockDim.x, ++nu) {
      float* gs = g.gates + row * 4 * H;
      g.hprev[row * H + u] = h[u];
      if (g.cell == NR_CELL_LSTM) {
        const float ig = sigm(xs[u] + gh[u]);
        const float fg = sigm(xs[H + u] + gh[H + u]);
        const float gg = tanhf(xs[2 * H + u] + gh[2 * H + u]);
        const float og = sigm(xs[3 * H + u] + gh[3 * H + u]);
        const float cc = fmaf(fg, c[u], ig * gg);
        g.cprev[row * H + u] = c[u];
        gs[u] = ig; gs[H + u] = fg; gs[2 * H + u] = gg; gs[3 * H + u] = og;
        cn[nu] = cc;
        hn[nu] = og * tanhf(cc);
      } else {
        const float rg = sigm(xs[u] + gh[u]);
        const float zg = sigm(xs[H + u] + gh[H + u]);
        const float ng = tanhf(fmaf(rg, gh[2 * H + u], xs[2 * H + u]));
        gs[u] = rg; gs[H + u] = zg; gs[2 * H + u] = ng; gs[3 * H + u] = gh[2 * H + u];
        cn[nu] = 0.f;
        hn[nu] = fmaf(zg, h[u] - ng, ng);     // (1 - z) n + z h
      }
    }
    __syncthreads();
    nu = 0;
    for (int u = tid; u < H; u += blockDim.x, ++nu) {
      h[u] = hn[nu];
      c[u] = cn[nu];
      if (t == len - 1) g.hout[b * g.ldho + u] = hn[nu];
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void rnn_bwd_kernel(RnnArgs g) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int H = g.H, G = g.cell == NR_CELL_LSTM ? 4 : 3, GH = G * H;
  float* dh = sm;           // [H]
  float* dc = dh + H;       // [H]  (LSTM: dc carried to t-1 ; GRU: dh direct path)
  float* dg = dc + H;       // [GH] recurrent-path gate grads
  int* red = reinterpret_cast<int*>(dg + GH);
  const int64_t b = blockIdx.x;
  const int tid = threadIdx.x;
  if (tid == 0) *red = 0;
  for (int u = tid; u < H; u += blockDim.x) {
    dh[u] = g.dhout[b * g.lddho + u];
    dc[u] = 0.f;
  }
  __syncthreads();
  const int len = seq_len(g, b, red);
  for (int t = len; t < g.N; ++t) {
    const int tt = g.reverse ? g.N - 1 - t : t;
    const int64_t row = b * g.N + tt;
    for (int r = tid; r < GH; r += blockDim.x) {
      g.dgi[row * g.lddg + r] = 0.f;
      if (g.dgh) g.dgh[row * g.lddg + r] = 0.f;
    }
  }
  for (int t = len - 1; t >= 0; --t) {
    const int tt = g.reverse ? g.N - 1 - t : t;
    const int64_t row = b * g.N + tt;
    const float* gs = g.gates + row * 4 * H;
    float* dgi = g.dgi + row * g.lddg;
    float* dgh = g.dgh ? g.dgh + row * g.lddg : nullptr;
    for (int u = tid; u < H; u += blockDim.x) {
      if (g.cell == NR_CELL_LSTM) {
        const float ig = gs[u], fg = gs[H + u], gg = gs[2 * H + u], og = gs[3 * H + u];
        const float cp = g.cprev[row * H + u];
        const float cc = fmaf(fg, cp, ig * gg);
        const float tc = tanhf(cc);
        const float dcc = dc[u] + dh[u] * og * (1.f - tc * tc);
        const float di = dcc * gg * ig * (1.f - ig);
        const float df = dcc * cp * fg * (1.f - fg);
        const float dgg = dcc * ig * (1.f - gg * gg);
        const float dog = dh[u] * tc * og * (1.f - og);
        dgi[u] = di; dgi[H + u] = df; dgi[2 * H + u] = dgg; dgi[3 * H + u] = dog;
        if (dgh) { dgh[u] = di; dgh[H + u] = df; dgh[2 * H + u] = dgg; dgh[3 * H + u] = dog; }
        dg[u] = di; dg[H + u] = df; dg[2 * H + u] = dgg; dg[3 * H + u] = dog;
        dc[u] = dcc * fg;                           // -> c_{t-1}
      } else {
        const float rg = gs[u], zg = gs[H + u], ng = gs[2 * H + u], ghn = gs[3 * H + u];
        const float hp = g.hprev[row * H + u];
        const float dn = dh[u] * (1.f - zg) * (1.f - ng * ng);
        const float dz = dh[u] * (hp - ng) * zg * (1.f - zg);
        const float dr = dn * ghn * rg * (1.f - rg);
        dgi[u] = dr; dgi[H + u] = dz; dgi[2 * H + u] = dn;
        dgh[u] = dr; dgh[H + u] = dz; dgh[2 * H + u] = dn * rg;
        dg[u] = dr; dg[H + u] = dz; dg[2 * H + u] = dn * rg;
        dc[u] = dh[u] * zg;                         // direct path to h_{t-1}
      }
    }
    __syncthreads();
    float nd[2];
    int nu = 0;
    for (int k = tid; k < H; k += blockDim.x, ++nu) {
      float acc = g.cell == NR_CELL_GRU ? dc[k] : 0.f;
      for (int r = 0; r < GH; ++r) acc = fmaf(dg[r], g.whh[(int64_t)r * H + k], acc);
      nd[nu] = acc;
    }
    __syncthreads();
    nu = 0;
    for (int k = tid; k < H; k += blockDim.x, ++nu) {
      dh[k] = nd[nu];
      if (g.cell == NR_CELL_GRU) dc[k] = 0.f;
    }
    __syncthreads();
  }
  if (g.dh0)
    for (int u = tid; u < H; u += blockDim.x) g.dh0[b * g.lddh0 + u] = dh[u];
}

// ---- weights-stationary forms for H = 150 (Manager.py:61): W_hh lives in registers for the whole
// sequence (one gate row per thread in the forward, 150 weights of one column per thread in the
// backward), so a step costs 150 FMAs against LDS-broadcast h (or dg) instead of 150 (or 600)
// dependent L2 loads.  One workgroup per sequence, G*H threads (LSTM 600, GRU 450).
// KR weights of each row in registers, the other H - KR in LDS as [k][row] (a wave reads 64
// consecutive floats: conflict-free): 600 LSTM rows at 3 waves/SIMD leave ~168 VGPRs per lane.
template <int H, int G, int KR>
__global__ __launch_bounds__(((G * H + 63) / 64) * 64) void rnn_fwd_reg_kernel(RnnArgs g) {
  constexpr int GH = G * H;
  constexpr int KL = H - KR;
  __shared__ __attribute__((aligned(16))) float h[H + 2];
  __shared__ float c[H];
  __shared__ float gh[GH];
  __shared__ float wl[KL > 0 ? KL * GH : 1];
  __shared__ int red;
  const int64_t b = blockIdx.x;
  const int tid = threadIdx.x;
  float w[KR];
  float bias = 0.f;
  if (tid < GH) {
#pragma unroll
    for (int k = 0; k < KR; ++k) w[k] = g.whh[(int64_t)k * GH + tid];   // W_hhᵀ [H][GH]: row tid of W_hh
    for (int k = KR; k < H; ++k) wl[(k - KR) * GH + tid] = g.whh[(int64_t)k * GH + tid];
    bias = g.bhh ? g.bhh[tid] : 0.f;
  }
  if (tid == 0) red = 0;
  if (tid < H) {
    float h0 = 0.f;
    if (g.h0) {
      const int64_t r = g.h0_idx ? g.h0_idx[b] : b;
      h0 = g.h0[r * g.ldh0 + tid];
    }
    h[tid] = h0;
    c[tid] = 0.f;
  }
  if (tid < 2) h[H + tid] = 0.f;
  __syncthreads();
  const int len = seq_len(g, b, &red);
  if (len == 0 && tid < H) g.hout[b * g.ldho + tid] = h[tid];   // all-zero mask row: h0
  // the input projections of step t + 1 are loaded during step t: the load latency (L2 / HBM, ~1 us)
  // otherwise sits on the sequential critical path of every step
  float xn[G];
  auto load_x = [&](int t) {
    const int tt = g.reverse ? g.N - 1 - t : t;
    const float* xs = g.gx + (b * g.N + tt) * g.ldgx + tid;
#pragma unroll
    for (int i = 0; i < G; ++i) xn[i] = xs[i * H];
  };
  if (tid < H && len > 0) load_x(0);
  for (int t = 0; t < g.N; ++t) {
    const int tt = g.reverse ? g.N - 1 - t : t;
    const int64_t row = b * g.N + tt;
    if (t >= len) {   // padded steps: zero what the backward GEMMs read
      for (int r = tid; r < 4 * H; r += blockDim.x) g.gates[row * 4 * H + r] = 0.f;
      if (tid < H) {
        g.hprev[row * H + tid] = 0.f;
        if (g.cprev) g.cprev[row * H + tid] = 0.f;
      }
      continue;
    }
    float xc[G];
#pragma unroll
    for (int i = 0; i < G; ++i) xc[i] = xn[i];
    if (tid < H && t + 1 < len) load_x(t + 1);
    if (tid < GH) {
      float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll
      for (int k = 0; k < KR; k += 4) {   // h is padded to a multiple of 4 with zeros
        const float4 hv = *reinterpret_cast<const float4*>(&h[k]);
        a0 = fmaf(w[k], hv.x, a0);
        if (k + 1 < KR) a1 = fmaf(w[k + 1], hv.y, a1);
        if (k + 2 < KR) a2 = fmaf(w[k + 2], hv.z, a2);
        if (k + 3 < KR) a3 = fmaf(w[k + 3], hv.w, a3);
        if ((k & 15) == 12) __builtin_amdgcn_sched_barrier(0);   // keep the h reads from all hoisting
      }
      if constexpr (KL > 0) {
        static_assert(KR % 4 == 0, "the LDS part of a row starts float4-aligned in h");
#pragma unroll 4
        for (int k = KR; k < H; k += 4) {   // h read as float4 (padded with zeros past H)
          const float4 hv = *reinterpret_cast<const float4*>(&h[k]);
          a0 = fmaf(wl[(k - KR) * GH + tid], hv.x, a0);
          if (k + 1 < H) a1 = fmaf(wl[(k + 1 - KR) * GH + tid], hv.y, a1);
          if (k + 2 < H) a2 = fmaf(wl[(k + 2 - KR) * GH + tid], hv.z, a2);
          if (k + 3 < H) a3 = fmaf(wl[(k + 3 - KR) * GH + tid], hv.w, a3);
        }
      }
      gh[tid] = bias + ((a0 + a1) + (a2 + a3));
    }
    __syncthreads();
    float hn = 0.f, cn = 0.f;
    if (tid < H) {
      const int u = tid;
      float* gs = g.gates + row * 4 * H;
      g.hprev[row * H + u] = h[u];
      if (G == 4) {
        const float ig = sigm(xc[0] + gh[u]);
        const float fg = sigm(xc[1] + gh[H + u]);
        const float gg = tanhf(xc[2] + gh[2 * H + u]);
        const float og = sigm(xc[3] + gh[3 * H + u]);
        const float cc = fmaf(fg, c[u], ig * gg);
        g.cprev[row * H + u] = c[u];
        gs[u] = ig; gs[H + u] = fg; gs[2 * H + u] = gg; gs[3 * H + u] = og;
        cn = cc;
        hn = og * tanhf(cc);
      } else {
        const float rg = sigm(xc[0] + gh[u]);
        const float zg = sigm(xc[1] + gh[H + u]);
        const float ng = tanhf(fmaf(rg, gh[2 * H + u], xc[2 % G]));
        gs[u] = rg; gs[H + u] = zg; gs[2 * H + u] = ng; gs[3 * H + u] = gh[2 * H + u];
        hn = fmaf(zg, h[u] - ng, ng);
      }
    }
    __syncthreads();
    if (tid < H) {
      h[tid] = hn;
      c[tid] = cn;
      if (t == len - 1) g.hout[b * g.ldho + tid] = hn;
    }
    __syncthreads();
  }
}

template <int H, int G>
__global__ __launch_bounds__(((G * H + 63) / 64) * 64) void rnn_bwd_reg_kernel(RnnArgs g) {
  constexpr int GH = G * H;
  __shared__ float dh[H];
  __shared__ float dc[H];
  __shared__ __attribute__((aligned(16))) float dg[GH + 4];
  __shared__ float ps[G][H];
  __shared__ int red;
  const int64_t b = blockIdx.x;
  const int tid = threadIdx.x;
  const int kcol = tid % H, part = tid / H;   // thread: column kcol of W_hh rows part*H .. part*H+H-1
  float w[H];
  if (tid < GH) {
#pragma unroll
    for (int i = 0; i < H; ++i) w[i] = g.whh[(int64_t)(part * H + i) * H + kcol];   // W_hh [GH][H]
  }
  if (tid == 0) red = 0;
  if (tid < H) {
    dh[tid] = g.dhout[b * g.lddho + tid];
    dc[tid] = 0.f;
  }
  if (tid < 4) dg[GH + tid] = 0.f;
  __syncthreads();
  const int len = seq_len(g, b, &red);
  for (int t = len; t < g.N; ++t) {
    const int tt = g.reverse ? g.N - 1 - t : t;
    const int64_t row = b * g.N + tt;
    for (int r = tid; r < GH; r += blockDim.x) {
      g.dgi[row * g.lddg + r] = 0.f;
      if (g.dgh) g.dgh[row * g.lddg + r] = 0.f;
    }
  }
  // the saved gates (and c_{t-1} / h_{t-1}) of step t - 1 are loaded during step t (off the
  // sequential critical path)
  float gn[4], pn = 0.f;
  auto load_g = [&](int t) {
    const int tt = g.reverse ? g.N - 1 - t : t;
    const int64_t row = b * g.N + tt;
    const float* gs = g.gates + row * 4 * H + tid;
#pragma unroll
    for (int i = 0; i < 4; ++i) gn[i] = gs[i * H];
    pn = G == 4 ? g.cprev[row * H + tid] : g.hprev[row * H + tid];
  };
  if (tid < H && len > 0) load_g(len - 1);
  for (int t = len - 1; t >= 0; --t) {
    const int tt = g.reverse ? g.N - 1 - t : t;
    const int64_t row = b * g.N + tt;
    float gc[4], pc = pn;
#pragma unroll
    for (int i = 0; i < 4; ++i) gc[i] = gn[i];
    if (tid < H && t > 0) load_g(t - 1);
    if (tid < H) {
      const int u = tid;
      float* dgi = g.dgi + row * g.lddg;
      float* dgh = g.dgh ? g.dgh + row * g.lddg : nullptr;
      if (G == 4) {
        const float ig = gc[0], fg = gc[1], gg = gc[2], og = gc[3];
        const float cp = pc;
        const float cc = fmaf(fg, cp, ig * gg);
        const float tc = tanhf(cc);
        const float dcc = dc[u] + dh[u] * og * (1.f - tc * tc);
        const float di = dcc * gg * ig * (1.f - ig);
        const float df = dcc * cp * fg * (1.f - fg);
        const float dgg = dcc * ig * (1.f - gg * gg);
        const float dog = dh[u] * tc * og * (1.f - og);
        dgi[u] = di; dgi[H + u] = df; dgi[2 * H + u] = dgg; dgi[3 * H + u] = dog;
        if (dgh) { dgh[u] = di; dgh[H + u] = df; dgh[2 * H + u] = dgg; dgh[3 * H + u] = dog; }
        dg[u] = di; dg[H + u] = df; dg[2 * H + u] = dgg; dg[3 * H + u] = dog;
        dc[u] = dcc * fg;
      } else {
        const float rg = gc[0], zg = gc[1], ng = gc[2], ghn = gc[3];
        const float hp = pc;
        const float dn = dh[u] * (1.f - zg) * (1.f - ng * ng);
        const float dz = dh[u] * (hp - ng) * zg * (1.f - zg);
        const float dr = dn * ghn * rg * (1.f - rg);
        dgi[u] = dr; dgi[H + u] = dz; dgi[2 * H + u] = dn;
        dgh[u] = dr; dgh[H + u] = dz; dgh[2 * H + u] = dn * rg;
        dg[u] = dr; dg[H + u] = dz; dg[2 * H + u] = dn * rg;
        dc[u] = dh[u] * zg;
      }
    }
    __syncthreads();
    if (tid < GH) {
      float a0 = 0.f, a1 = 0.f;
      const float* d = dg + part * H;
#pragma unroll
      for (int i = 0; i < H; i += 2) {
        a0 = fmaf(d[i], w[i], a0);
        if (i + 1 < H) a1 = fmaf(d[i + 1], w[i + 1], a1);
        if ((i & 15) == 14) __builtin_amdgcn_sched_barrier(0);
      }
      ps[part][kcol] = a0 + a1;
    }
    __syncthreads();
    if (tid < H) {
      float acc = G == 3 ? dc[tid] : 0.f;
#pragma unroll
      for (int p = 0; p < G; ++p) acc += ps[p][tid];
      dh[tid] = acc;
      if (G == 3) dc[tid] = 0.f;
    }
    __syncthreads();
  }
  if (g.dh0 && tid < H) g.dh0[b * g.lddh0 + tid] = dh[tid];
}

size_t rnn_smem(int cell, int H) { return (size_t)(2 * H + (cell == NR_CELL_LSTM ? 4 : 3) * H + 4) * sizeof(float); }

}  // namespace

extern "C" int nr_rnn_fwd(int32_t cell, const float* gx, int64_t ldgx, const float* whh_t, const float* bhh,
                          const float* h0, int64_t ldh0, const int64_t* h0_idx, const void* mask,
                          int32_t mask_dtype, int32_t reverse, int64_t B, int32_t N, int32_t H, float* gates,
                          float* hprev, float* cprev, float* hout, int64_t ldho, hipStream_t stream) {
  if ((cell != NR_CELL_LSTM && cell != NR_CELL_GRU) || B < 0 || N < 1 || H < 1 || H > 512) return NR_EINVAL(0);
  if (!gx || !whh_t || !gates || !hprev || !hout || (cell == NR_CELL_LSTM && !cprev)) return NR_EINVAL(1);
  if (B == 0) return NR_OK;
  RnnArgs g{};
  g.cell = cell; g.gx = gx; g.ldgx = ldgx; g.whh = whh_t; g.bhh = bhh; g.h0 = h0; g.ldh0 = ldh0;
  g.h0_idx = h0_idx; g.mask = mask; g.mask_dt = mask_dtype; g.reverse = reverse; g.B = B; g.N = N; g.H = H;
  g.gates = gates; g.hprev = hprev; g.cprev = cprev; g.hout = hout; g.ldho = ldho;
  if (H == 150) {
    if (cell == NR_CELL_LSTM) hipLaunchKernelGGL((rnn_fwd_reg_kernel<150, 4, 88>), dim3((unsigned)B), dim3(640), 0, stream, g);
    else hipLaunchKernelGGL((rnn_fwd_reg_kernel<150, 3, 150>), dim3((unsigned)B), dim3(512), 0, stream, g);
    NR_LAUNCH_CHECK();
    return NR_OK;
  }
  hipLaunchKernelGGL(rnn_fwd_kernel, dim3((unsigned)B), dim3(256), rnn_smem(cell, H), stream, g);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

extern "C" int nr_rnn_bwd(int32_t cell, const float* whh, const float* gates, const float* hprev,
                          const float* cprev, const void* mask, int32_t mask_dtype, int32_t reverse, int64_t B,
                          int32_t N, int32_t H, const float* dhout, int64_t lddho, float* dgi, float* dgh,
                          int64_t lddg, float* dh0, int64_t lddh0, hipStream_t stream) {
  if ((cell != NR_CELL_LSTM && cell != NR_CELL_GRU) || B < 0 || N < 1 || H < 1 || H > 512) return NR_EINVAL(0);
  if (!whh || !gates || !hprev || !dhout || !dgi || (cell == NR_CELL_LSTM && !cprev) ||
      (cell == NR_CELL_GRU && !dgh))
    return NR_EINVAL(1);
  if (B == 0) return NR_OK;
  RnnArgs g{};
  g.cell = cell; g.whh = whh; g.gates = const_cast<float*>(gates); g.hprev = const_cast<float*>(hprev);
  g.cprev = const_cast<float*>(cprev); g.mask = mask; g.mask_dt = mask_dtype; g.reverse = reverse; g.B = B;
  g.N = N; g.H = H; g.dhout = dhout; g.lddho = lddho; g.dgi = dgi; g.dgh = dgh; g.lddg = lddg; g.dh0 = dh0;
  g.lddh0 = lddh0;
  if (H == 150) {
    if (cell == NR_CELL_LSTM) hipLaunchKernelGGL((rnn_bwd_reg_kernel<150, 4>), dim3((unsigned)B), dim3(640), 0, stream, g);
    else hipLaunchKernelGGL((rnn_bwd_reg_kernel<150, 3>), dim3((unsigned)B), dim3(512), 0, stream, g);
    NR_LAUNCH_CHECK();
    return NR_OK;
  }
  hipLaunchKernelGGL(rnn_bwd_kernel, dim3((unsigned)B), dim3(256), rnn_smem(cell, H), stream, g);
  NR_LAUNCH_CHECK();
  return NR_OK;
}
