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

__device__ __forceinline__ float nr_wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float nr_wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Counter-based RNG for dropout: a stateless hash of (seed, offset + element index), so
// forward and backward regenerate the same keep mask without storing it.
__device__ __forceinline__ uint32_t nr_hash3(uint64_t seed, uint64_t ctr) {
  uint64_t z = seed * 0x9E3779B97F4A7C15ull + ctr * 0xD1B54A32D192ED03ull + 0x632BE59BD9B4E019ull;
  z ^= z >> 30; z *= 0xBF58476D1CE4E5B9ull;
  z ^= z >> 27; z *= 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (uint32_t)(z >> 32);
}

__device__ __forceinline__ bool nr_dropout_keep(uint64_t seed, uint64_t ctr, float p) {
  // keep with probability 1 - p
  return (float)(nr_hash3(seed, ctr) >> 8) * (1.0f / 16777216.0f) >= p;
}
