// Shared helpers for the newsrec HIP kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define NR_WAVE 64

// Return codes of the C ABI: 0 = ok, negative = error.  -1000 - x : invalid argument x.
#define NR_OK 0
#define NR_EINVAL(x) (-1000 - (x))

#define NR_LAUNCH_CHECK()                                   \
  do {                                                      \
    hipError_t e__ = hipGetLastError();                     \
    if (e__ != hipSuccess) return -(int)e__;                \
  } while (0)

// Mask element types accepted by the kernels (the reference feeds i64 token masks and
// an f64 history mask; see utils/MIND.py:330-350).
enum nr_mask_dtype { NR_MASK_U8 = 0, NR_MASK_I64 = 1, NR_MASK_F64 = 2, NR_MASK_F32 = 3 };

__device__ __forceinline__ bool nr_mask_at(const void* m, int dt, int64_t i) {
  switch (dt) {
    case NR_MASK_U8: return ((const uint8_t*)m)[i] != 0;
    case NR_MASK_I64: return ((const int64_t*)m)[i] != 0;
    case NR_MASK_F64: return ((const double*)m)[i] != 0.0;
    default: return ((const float*)m)[i] != 0.0f;
  }
}

// Wave-wide all-reduce without the LDS crossbar: DPP inside each 16-lane row (quad_perm
// [1,0,3,2], quad_perm [2,3,0,1], row_half_mirror, row_mirror), then the gfx950 row swaps
// v_permlane16_swap / v_permlane32_swap.  Every lane ends with the full result.
__device__ __forceinline__ float nr_dpp(float v, int ctrl_sel) {
  const int x = __builtin_bit_cast(int, v);
  int r;
  switch (ctrl_sel) {
    case 0: r = __builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, false); break;    // quad_perm [1,0,3,2]
    case 1: r = __builtin_amdgcn_mov_dpp(x, 0x4E, 0xF, 0xF, false); break;    // quad_perm [2,3,0,1]
    case 2: r = __builtin_amdgcn_mov_dpp(x, 0x141, 0xF, 0xF, false); break;   // row_half_mirror
    default: r = __builtin_amdgcn_mov_dpp(x, 0x140, 0xF, 0xF, false); break;  // row_mirror
  }
  return __builtin_bit_cast(float, r);
}

__device__ __forceinline__ float nr_wave_sum(float v) {
  v += nr_dpp(v, 0);
  v += nr_dpp(v, 1);
  v += nr_dpp(v, 2);
  v += nr_dpp(v, 3);
  {
    const unsigned x = __builtin_bit_cast(unsigned, v);
    auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    v = __builtin_bit_cast(float, (unsigned)r[0]) + __builtin_bit_cast(float, (unsigned)r[1]);
  }
  {
    const unsigned x = __builtin_bit_cast(unsigned, v);
    auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    v = __builtin_bit_cast(float, (unsigned)r[0]) + __builtin_bit_cast(float, (unsigned)r[1]);
  }
  return v;
}

__device__ __forceinline__ float nr_wave_max(float v) {
  v = fmaxf(v, nr_dpp(v, 0));
  v = fmaxf(v, nr_dpp(v, 1));
  v = fmaxf(v, nr_dpp(v, 2));
  v = fmaxf(v, nr_dpp(v, 3));
  {
    const unsigned x = __builtin_bit_cast(unsigned, v);
    auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    v = fmaxf(__builtin_bit_cast(float, (unsigned)r[0]), __builtin_bit_cast(float, (unsigned)r[1]));
  }
  {
    const unsigned x = __builtin_bit_cast(unsigned, v);
    auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    v = fmaxf(__builtin_bit_cast(float, (unsigned)r[0]), __builtin_bit_cast(float, (unsigned)r[1]));
  }
  return v;
}

// Counter-based RNG for dropout.  Each call derives a 32-bit key from (seed, offset) on the
// host, or in the kernel from a device-resident (seed, offset) pair when the call sits in a
// replayed graph (splitmix64, nr_dropout_key); each element's keep bit is a 32-bit hash (lowbias32) of
// key + index, compared with a 32-bit threshold.  Stateless: the backward regenerates the
// forward's mask exactly, nothing is stored.
__host__ __device__ static inline uint32_t nr_dropout_key(uint64_t seed, uint64_t offset) {
  uint64_t z = seed * 0x9E3779B97F4A7C15ull + offset * 0xD1B54A32D192ED03ull + 0x632BE59BD9B4E019ull;
  z ^= z >> 30; z *= 0xBF58476D1CE4E5B9ull;
  z ^= z >> 27; z *= 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (uint32_t)(z >> 32);
}

static inline uint32_t nr_dropout_threshold(float p) {   // drop iff hash < threshold
  const double t = (double)p * 4294967296.0;
  return t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
}

__device__ __forceinline__ uint32_t nr_hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7FEB352Du;
  x ^= x >> 15; x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

__device__ __forceinline__ bool nr_dropout_keep(uint32_t key, uint32_t elem, uint32_t thresh) {
  return nr_hash32(key + elem * 0x9E3779B1u) >= thresh;
}

// Exact (erf) GELU of transformers' "gelu" activation (BertIntermediate) and its derivative.
__device__ __forceinline__ float nr_gelu(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float nr_gelu_grad(float x) {
  const float cdf = 0.5f * (1.f + erff(x * 0.70710678118654752f));
  return cdf + x * 0.39894228040143268f * __expf(-0.5f * x * x);
}
