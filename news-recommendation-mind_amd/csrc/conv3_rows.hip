// Distinct-row k = 3 convolution of the CNN news encoder (models/Encoders/CNN.py:12-17,41-42).
//
// Conv1d(E -> H, k = 3, pad = 1) over gathered word rows is linear in each tap, so it commutes with
// the gather: with P[u] = [W_0 table[u] | W_1 table[u] | W_2 table[u]] computed ONCE per distinct
// word row u of the batch (one GEMM over U rows instead of a K = 3E GEMM over T tokens),
//   C[t] = ReLU(b + sum_j P[inv[t + j - 1]][tap j])     (zero taps outside the title)
// is a three-row gather-add per token.  The backward mirrors it (nr_segment_rows_sum_conv3 sums
// the shifted dC rows per distinct row; the table dgrad and the conv wgrad are then GEMMs over U).
#include "common.h"
#include "../../include/newsrec_hip.h"

namespace {

// one thread per (token, float4 column); consecutive threads walk one token's columns
__global__ __launch_bounds__(256) void conv3_rows_fwd_kernel(const float* __restrict__ P, int64_t ldp, int tw4,
                                                             int H, const int64_t* __restrict__ inv, int64_t T, int L,
                                                             const float* __restrict__ bias, int relu,
                                                             float* __restrict__ out, int64_t ldo) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= T * tw4) return;
  const int64_t t = g / tw4;
  const int c4 = (int)(g - t * tw4);
  const int pos = (int)(t % L);
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int p2 = pos + j - 1;
    if (p2 < 0 || p2 >= L) continue;
    const int64_t r = inv[t + j - 1];
    const float4 v = reinterpret_cast<const float4*>(P + r * ldp)[j * tw4 + c4];
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  const int h = 4 * c4;
  float e[4] = {s.x, s.y, s.z, s.w};
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    if (h + u < H) {
      float x = e[u] + (bias ? bias[h + u] : 0.f);
      e[u] = relu ? fmaxf(x, 0.f) : x;
    } else {
      e[u] = 0.f;   // padded columns: exact zeros (the next GEMM contracts over them)
    }
  }
  reinterpret_cast<float4*>(out + t * ldo)[c4] = make_float4(e[0], e[1], e[2], e[3]);
}

}  // namespace

extern "C" int nr_conv3_rows_fwd(const float* P, int64_t ldp, int32_t tap_width, int32_t H, const int64_t* inv,
                                 int64_t T, int32_t L, const float* bias, int32_t relu, float* out, int64_t ldo,
                                 hipStream_t stream) {
  if (tap_width < 4 || (tap_width & 3) || H < 1 || H > tap_width || L < 1 || T < 0 || (T % L) || (ldp & 3) ||
      (ldo & 3) || ldp < 3 * tap_width || ldo < tap_width)
    return NR_EINVAL(0);
  if (!P || !inv || !out) return NR_EINVAL(1);
  if ((reinterpret_cast<uintptr_t>(P) & 15) || (reinterpret_cast<uintptr_t>(out) & 15)) return NR_EINVAL(2);
  if (T == 0) return NR_OK;
  const int tw4 = tap_width / 4;
  const int64_t n = T * tw4;
  hipLaunchKernelGGL(conv3_rows_fwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, P, ldp, tw4, H,
                     inv, T, L, bias, relu, out, ldo);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

// ---- the distinct-row encoder's weight operands, one launch each way (the step's weights change
// every optimizer step, so they are re-laid out every step: one kernel instead of a permute copy
// and three pads, and one for their gradients instead of the matching slice / permute copies)
namespace {

__global__ __launch_bounds__(256) void cnn_pack_kernel(const float* __restrict__ cw, const float* __restrict__ wq,
                                                       const float* __restrict__ bq, int H, int E, int Hp,
                                                       float* __restrict__ w3t, float* __restrict__ wqp,
                                                       float* __restrict__ bqp, float* __restrict__ w3tt) {
  const int64_t n3 = (int64_t)3 * Hp * E, nq = (int64_t)Hp * Hp;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n3 + nq + Hp;
       i += (int64_t)gridDim.x * blockDim.x) {
    if (i < n3) {   // w3t[tap*Hp + h][e] = conv.weight[h][e][tap]; w3tt its transpose [e][tap*Hp + h]
      const int64_t r = i / E, e = i - r * E;
      const int tap = (int)(r / Hp), h = (int)(r - (int64_t)tap * Hp);
      const float x = h < H ? cw[((int64_t)h * E + e) * 3 + tap] : 0.f;
      w3t[i] = x;
      if (w3tt) w3tt[e * 3 * Hp + r] = x;
    } else if (i < n3 + nq) {
      const int64_t k = i - n3;
      const int r = (int)(k / Hp), c = (int)(k - (int64_t)r * Hp);
      wqp[k] = (r < H && c < H) ? wq[(int64_t)r * H + c] : 0.f;
    } else {
      const int h = (int)(i - n3 - nq);
      bqp[h] = h < H ? bq[h] : 0.f;
    }
  }
}

__global__ __launch_bounds__(256) void cnn_unpack_kernel(const float* __restrict__ dw3t, const float* __restrict__ dwqp,
                                                         const float* __restrict__ dbqp, int H, int E, int Hp,
                                                         float* __restrict__ dcw, float* __restrict__ dwq,
                                                         float* __restrict__ dbq) {
  const int64_t n3 = (int64_t)3 * H * E, nq = (int64_t)H * H;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n3 + nq + H;
       i += (int64_t)gridDim.x * blockDim.x) {
    if (i < n3) {   // dconv.weight[h][e][tap] = dw3t[tap*Hp + h][e]
      const int64_t he = i / 3;
      const int tap = (int)(i - he * 3);
      const int64_t h = he / E, e = he - h * E;
      dcw[i] = dw3t[((int64_t)tap * Hp + h) * E + e];
    } else if (i < n3 + nq) {
      const int64_t k = i - n3;
      const int r = (int)(k / H), c = (int)(k - (int64_t)r * H);
      dwq[k] = dwqp[(int64_t)r * Hp + c];
    } else {
      const int h = (int)(i - n3 - nq);
      dbq[h] = dbqp[h];
    }
  }
}

}  // namespace

extern "C" int nr_cnn_pack_weights(const float* conv_w, const float* wq, const float* bq, int32_t H, int32_t E,
                                   int32_t Hp, float* w3t, float* wqp, float* bqp, float* w3tt, hipStream_t stream) {
  if (H < 1 || E < 1 || Hp < H) return NR_EINVAL(0);
  if (!conv_w || !wq || !bq || !w3t || !wqp || !bqp) return NR_EINVAL(1);
  hipLaunchKernelGGL(cnn_pack_kernel, dim3(1024), dim3(256), 0, stream, conv_w, wq, bq, H, E, Hp, w3t, wqp, bqp,
                     w3tt);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

extern "C" int nr_cnn_unpack_grads(const float* dw3t, const float* dwqp, const float* dbqp, int32_t H, int32_t E,
                                   int32_t Hp, float* dconv_w, float* dwq, float* dbq, hipStream_t stream) {
  if (H < 1 || E < 1 || Hp < H) return NR_EINVAL(0);
  if (!dw3t || !dwqp || !dbqp || !dconv_w || !dwq || !dbq) return NR_EINVAL(1);
  hipLaunchKernelGGL(cnn_unpack_kernel, dim3(1024), dim3(256), 0, stream, dw3t, dwqp, dbqp, H, E, Hp, dconv_w, dwq, dbq);
  NR_LAUNCH_CHECK();
  return NR_OK;
}
