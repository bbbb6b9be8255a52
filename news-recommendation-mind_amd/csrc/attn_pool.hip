// Learned-query attention pooling over a short sequence, with the optional LayerNorm and
// dropout that precede it in the MHA news encoder:
//
//   Z_l   = Dropout(LayerNorm(X_l))            (MHA.py:37; identity when no LN / p = 0)
//   s_l   = scale * q · K_l,  K = Z (tied) or a separate key matrix
//   p     = XSoftmax(s, mask)                  (Attention.py:56-80; masked -> exactly 0)
//   out   = Σ_l p_l Z_l                        (scaled_dp_attention, Attention.py:5-30)
//
// Call sites it replaces:
//   MHA_Encoder.forward   MHA.py:37-38   (LN + dropout, tied key, query_words, token mask)
//   MHA_User_Encoder      MHA.py:72      (tied key, query_news, history mask)
//   Attention_Pooling     Pooling.py:22-24
//   CNN_Encoder           CNN.py:46      (key = tanh(W c + b) from a separate GEMM)
//
// One 256-thread workgroup per sequence: LN statistics by wave reductions, Z staged in LDS,
// scores one wave per row, the softmax in one wave (lane = position), the weighted sum one
// thread per feature.  Backward recomputes Z from X and the saved (mean, rstd, p), and
// produces dX (through LN and dropout), dK (optionally through tanh'), and atomically
// accumulates dq, dgamma, dbeta.
#include "common.h"
#include "../../include/newsrec_hip.h"

namespace {

struct PoolArgs {
  const float* x; int64_t ldx;
  const float* key; int64_t ldk;          // NULL: tied (key = Z)
  const float* q;
  const void* mask; int mask_dt;
  const float* gamma; const float* beta;  // NULL: no LayerNorm
  float eps;
  float p_drop; uint64_t seed; uint64_t offset;
  uint32_t dkey, dthresh;                  // dropout key / threshold derived on the host
  const uint64_t* rng;                     // device (seed, offset base): key derived in the kernel
  int64_t nseq; int L; int D; float scale;
  float* out; int64_t ldo;
  float* zout; int64_t ldz;                // optional: write Z (the encoder's token output)
  const float* dz; int64_t lddz;           // optional: upstream grad of Z (bwd)
  float* stats;                            // [nseq*L][2] (mean, rstd) when LN
  float* probs;                            // [nseq*L]
  // backward
  const float* dout; int64_t lddo;
  float* dx; int64_t lddx;
  float* dk; int64_t lddk; int key_tanh;
  float* dq; float* dgamma; float* dbeta;
};

__device__ __forceinline__ float drop_scale(const PoolArgs& g, int64_t elem) {
  if (g.p_drop <= 0.f) return 1.f;
  return nr_dropout_keep(g.dkey, (uint32_t)elem, g.dthresh) ? 1.f / (1.f - g.p_drop) : 0.f;
}

// Stage Z rows of sequence `seq` in LDS (zs[l*D + d]); writes LN stats when `save`.
__device__ void stage_z(const PoolArgs& g, int64_t seq, float* zs, bool save, bool from_stats) {
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  for (int l = w; l < g.L; l += 4) {
    const int64_t row = seq * g.L + l;
    const float* x = g.x + row * g.ldx;
    if (g.gamma) {
      float mean, rstd;
      if (from_stats) {
        mean = g.stats[2 * row];
        rstd = g.stats[2 * row + 1];
      } else {
        float s = 0.f;
        for (int d = lane; d < g.D; d += 64) s += x[d];
        mean = nr_wave_sum(s) / g.D;
        float v = 0.f;
        for (int d = lane; d < g.D; d += 64) { const float c = x[d] - mean; v = fmaf(c, c, v); }
        rstd = rsqrtf(nr_wave_sum(v) / g.D + g.eps);
        if (save && lane == 0) { g.stats[2 * row] = mean; g.stats[2 * row + 1] = rstd; }
      }
      for (int d = lane; d < g.D; d += 64) {
        const float y = (x[d] - mean) * rstd * g.gamma[d] + g.beta[d];
        zs[l * g.D + d] = y * drop_scale(g, row * g.D + d);
      }
    } else {
      for (int d = lane; d < g.D; d += 64) zs[l * g.D + d] = x[d] * drop_scale(g, row * g.D + d);
    }
  }
}

__device__ __forceinline__ const float* key_row(const PoolArgs& g, const float* zs, int64_t seq, int l) {
  return g.key ? g.key + (seq * g.L + l) * g.ldk : zs + l * g.D;
}

__global__ __launch_bounds__(256) void attn_pool_fwd_kernel(PoolArgs g) {
  if (g.rng) g.dkey = nr_dropout_key(g.rng[0], g.rng[1] + g.offset);   // graph-replay RNG
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* zs = smem;                       // [L][D]
  float* sc = smem + (size_t)g.L * g.D;   // [64]
  const int64_t seq = blockIdx.x;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  stage_z(g, seq, zs, true, false);
  __syncthreads();
  if (g.zout)
    for (int l = w; l < g.L; l += 4)
      for (int d = lane; d < g.D; d += 64) g.zout[(seq * g.L + l) * g.ldz + d] = zs[l * g.D + d];
  for (int l = w; l < g.L; l += 4) {
    const float* k = key_row(g, zs, seq, l);
    float s = 0.f;
    for (int d = lane; d < g.D; d += 64) s = fmaf(g.q[d], k[d], s);
    s = nr_wave_sum(s);
    if (lane == 0) sc[l] = s * g.scale;
  }
  __syncthreads();
  if (w == 0) {
    const int l = lane;
    const bool keep = l < g.L && nr_mask_at(g.mask, g.mask_dt, seq * g.L + l);
    const float v = keep ? sc[l] : -INFINITY;
    const float mx = nr_wave_max(v);
    const float e = keep ? __expf(v - mx) : 0.f;
    const float sum = nr_wave_sum(e);
    const float p = sum > 0.f ? e / sum : 0.f;
    if (l < g.L) {
      sc[l] = p;
      if (g.probs) g.probs[seq * g.L + l] = p;
    }
  }
  __syncthreads();
  for (int d = tid; d < g.D; d += 256) {
    float acc = 0.f;
    for (int l = 0; l < g.L; ++l) acc = fmaf(sc[l], zs[l * g.D + d], acc);
    g.out[seq * g.ldo + d] = acc;
  }
}

__global__ __launch_bounds__(256) void attn_pool_bwd_kernel(PoolArgs g) {
  if (g.rng) g.dkey = nr_dropout_key(g.rng[0], g.rng[1] + g.offset);   // graph-replay RNG
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* zs = smem;                         // [L][D]
  float* ps = smem + (size_t)g.L * g.D;     // [64] p
  float* ds = ps + 64;                      // [64] dp then ds
  float* dgb = ds + 64;                     // [2][D] block partial dgamma / dbeta
  const int64_t seq = blockIdx.x;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  stage_z(g, seq, zs, false, true);
  if (tid < 64) ps[tid] = tid < g.L ? g.probs[seq * g.L + tid] : 0.f;
  if (g.gamma)
    for (int d = tid; d < 2 * g.D; d += 256) dgb[d] = 0.f;
  __syncthreads();
  const float* dout = g.dout + seq * g.lddo;
  // dp_l = dout . Z_l
  for (int l = w; l < g.L; l += 4) {
    float s = 0.f;
    for (int d = lane; d < g.D; d += 64) s = fmaf(dout[d], zs[l * g.D + d], s);
    s = nr_wave_sum(s);
    if (lane == 0) ds[l] = s;
  }
  __syncthreads();
  if (w == 0) {
    const int l = lane;
    const float p = ps[l];
    const float dp = l < g.L ? ds[l] : 0.f;
    const float r = nr_wave_sum(p * dp);
    if (l < g.L) ds[l] = p * (dp - r) * g.scale;   // scale folded in: d(q·K) = scale * ds_raw
  }
  __syncthreads();
  // dq_d = Σ_l ds_l K_l[d];  separate key: dK_l[d] = ds_l q[d] (· (1 - K²) for a tanh key)
  for (int d = tid; d < g.D; d += 256) {
    float acc = 0.f;
    for (int l = 0; l < g.L; ++l) {
      const float kv = g.key ? g.key[(seq * g.L + l) * g.ldk + d] : zs[l * g.D + d];
      acc = fmaf(ds[l], kv, acc);
      if (g.key) {
        float dkv = ds[l] * g.q[d];
        if (g.key_tanh) dkv *= (1.f - kv * kv);
        g.dk[(seq * g.L + l) * g.lddk + d] = dkv;
      }
    }
    atomicAdd(&g.dq[d], acc);
  }
  // dZ, dropout, LayerNorm backward: one wave per row
  for (int l = w; l < g.L; l += 4) {
    const int64_t row = seq * g.L + l;
    const float pl = ps[l], dsl = ds[l];
    float* dxr = g.dx + row * g.lddx;
    if (!g.gamma) {
      for (int d = lane; d < g.D; d += 64) {
        float dz = pl * dout[d];
        if (!g.key) dz = fmaf(dsl, g.q[d], dz);
        if (g.dz) dz += g.dz[row * g.lddz + d];
        dxr[d] = dz * drop_scale(g, row * g.D + d);
      }
      continue;
    }
    const float* x = g.x + row * g.ldx;
    const float mean = g.stats[2 * row], rstd = g.stats[2 * row + 1];
    float sg = 0.f, sgx = 0.f;
    for (int d = lane; d < g.D; d += 64) {
      float dz = pl * dout[d];
      if (!g.key) dz = fmaf(dsl, g.q[d], dz);
      if (g.dz) dz += g.dz[row * g.lddz + d];
      const float dy = dz * drop_scale(g, row * g.D + d);   // grad wrt the LN output
      const float xh = (x[d] - mean) * rstd;
      const float gg = dy * g.gamma[d];
      sg += gg;
      sgx = fmaf(gg, xh, sgx);
      atomicAdd(&dgb[d], dy * xh);
      atomicAdd(&dgb[g.D + d], dy);
      dxr[d] = dy;                                            // stash dy, finished below
    }
    sg = nr_wave_sum(sg) / g.D;
    sgx = nr_wave_sum(sgx) / g.D;
    for (int d = lane; d < g.D; d += 64) {
      const float xh = (x[d] - mean) * rstd;
      dxr[d] = rstd * (dxr[d] * g.gamma[d] - sg - xh * sgx);
    }
  }
  if (g.gamma) {
    __syncthreads();
    for (int d = tid; d < g.D; d += 256) {
      atomicAdd(&g.dgamma[d], dgb[d]);
      atomicAdd(&g.dbeta[d], dgb[g.D + d]);
    }
  }
}

size_t smem_fwd(int L, int D) { return ((size_t)L * D + 64) * sizeof(float); }
size_t smem_bwd(int L, int D) { return ((size_t)L * D + 128 + 2 * (size_t)D) * sizeof(float); }

}  // namespace

extern "C" int nr_attn_pool_fwd(const float* x, int64_t ldx, const float* key, int64_t ldk,
                                const float* q, const void* mask, int32_t mask_dtype,
                                const float* gamma, const float* beta, float eps, float p_drop,
                                uint64_t seed, uint64_t offset, const uint64_t* rng, int64_t nseq, int32_t L, int32_t D,
                                float scale, float* out, int64_t ldo, float* zout, int64_t ldz,
                                float* stats, float* probs, hipStream_t stream) {
  if (L < 1 || L > 64 || D < 1) return NR_EINVAL(0);
  if (!x || !q || !mask || !out || !probs) return NR_EINVAL(1);
  if (gamma && (!beta || !stats)) return NR_EINVAL(2);
  if (smem_bwd(L, D) > 160 * 1024) return NR_EINVAL(3);
  if (nseq == 0) return NR_OK;
  PoolArgs g{};
  g.x = x; g.ldx = ldx; g.key = key; g.ldk = ldk; g.q = q; g.mask = mask; g.mask_dt = mask_dtype;
  g.gamma = gamma; g.beta = beta; g.eps = eps; g.p_drop = p_drop; g.seed = seed; g.offset = offset;
  g.dkey = nr_dropout_key(seed, offset); g.dthresh = nr_dropout_threshold(p_drop); g.rng = rng;
  g.nseq = nseq; g.L = L; g.D = D; g.scale = scale; g.out = out; g.ldo = ldo; g.stats = stats;
  g.probs = probs; g.zout = zout; g.ldz = ldz;
  if (smem_fwd(L, D) > 64 * 1024)
    hipFuncSetAttribute((const void*)attn_pool_fwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)smem_fwd(L, D));
  hipLaunchKernelGGL(attn_pool_fwd_kernel, dim3((unsigned)nseq), dim3(256), smem_fwd(L, D), stream, g);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

extern "C" int nr_attn_pool_bwd(const float* x, int64_t ldx, const float* key, int64_t ldk,
                                const float* q, const void* mask, int32_t mask_dtype,
                                const float* gamma, const float* beta, float p_drop, uint64_t seed,
                                uint64_t offset, const uint64_t* rng, int64_t nseq, int32_t L, int32_t D,
                                float scale, const float* stats, const float* probs, const float* dout,
                                int64_t lddo, const float* dz, int64_t lddz, float* dx, int64_t lddx,
                                float* dk, int64_t lddk,
                                int32_t key_tanh, float* dq, float* dgamma, float* dbeta,
                                hipStream_t stream) {
  if (L < 1 || L > 64 || D < 1) return NR_EINVAL(0);
  if (!x || !q || !mask || !probs || !dout || !dx || !dq) return NR_EINVAL(1);
  if (gamma && (!beta || !stats || !dgamma || !dbeta)) return NR_EINVAL(2);
  if (key && !dk) return NR_EINVAL(3);
  if (smem_bwd(L, D) > 160 * 1024) return NR_EINVAL(4);
  if (nseq == 0) return NR_OK;
  PoolArgs g{};
  g.x = x; g.ldx = ldx; g.key = key; g.ldk = ldk; g.q = q; g.mask = mask; g.mask_dt = mask_dtype;
  g.gamma = gamma; g.beta = beta; g.p_drop = p_drop; g.seed = seed; g.offset = offset;
  g.dkey = nr_dropout_key(seed, offset); g.dthresh = nr_dropout_threshold(p_drop); g.rng = rng;
  g.nseq = nseq; g.L = L; g.D = D; g.scale = scale; g.stats = const_cast<float*>(stats);
  g.probs = const_cast<float*>(probs); g.dout = dout; g.lddo = lddo; g.dx = dx; g.lddx = lddx;
  g.dk = dk; g.lddk = lddk; g.key_tanh = key_tanh; g.dq = dq; g.dgamma = dgamma; g.dbeta = dbeta;
  g.dz = dz; g.lddz = lddz;
  if (smem_bwd(L, D) > 64 * 1024)
    hipFuncSetAttribute((const void*)attn_pool_bwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)smem_bwd(L, D));
  hipLaunchKernelGGL(attn_pool_bwd_kernel, dim3((unsigned)nseq), dim3(256), smem_bwd(L, D), stream, g);
  NR_LAUNCH_CHECK();
  return NR_OK;
}
