// MFMA products over per-lane fp32 fragments in a selectable arithmetic, shared by the fused
// per-title kernels (mha_pool.hip, cnn_keypool.hip).
#pragma once
#include "common.h"
#include "gemm_fast_common.h"   // bf16 split helpers (nrfast::split2 / pk_bf16), f32x16, bf16x8

namespace {

// ---- Attention products in the caller's GEMM arithmetic (MPArgs::np, from nr_gemm_precision):
// NP = 0: v_mfma_f32_32x32x2_f32 (exact fp32 products); NP = 3: bf16x6 (three bf16 terms per fp32
// value, six v_mfma_f32_32x32x16_bf16 products -- the GEMMs' fp32-class arithmetic at 2.7x the f32
// MFMA's rate here); NP = 1: bf16 (one product).  A 32x32x16 bf16 operand gives lane (c, h) eight
// k-slots 8h .. 8h + 7; every product below feeds the lane eight consecutive values of a register
// array it already holds in the f32 form's k order, so the C layouts are the f32 form's.
template <int NP>
struct Planes {
  bf16x8 v[NP];
};

template <int NP>
__device__ __forceinline__ Planes<NP> planes8(const float* x) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  uint32_t h[4], m[4], l[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    if constexpr (NP == 1) {
      h[u] = nrfast::pk_bf16(x[2 * u], x[2 * u + 1]);
    } else {
      nrfast::split2(x[2 * u], x[2 * u + 1], h[u], m[u], l[u]);
    }
  }
  Planes<NP> r;
  r.v[0] = __builtin_bit_cast(bf16x8, (u32x4){h[0], h[1], h[2], h[3]});
  if constexpr (NP == 3) {
    r.v[1] = __builtin_bit_cast(bf16x8, (u32x4){m[0], m[1], m[2], m[3]});
    r.v[2] = __builtin_bit_cast(bf16x8, (u32x4){l[0], l[1], l[2], l[3]});
  }
  return r;
}

// acc += A B over one 16-deep step (smallest terms first)
template <int NP>
__device__ __forceinline__ void mfma_x(f32x16& acc, const Planes<NP>& a, const Planes<NP>& b) {
  if constexpr (NP == 3) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.v[2], b.v[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.v[1], b.v[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.v[0], b.v[2], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.v[1], b.v[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.v[0], b.v[1], acc, 0, 0, 0);
  }
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.v[0], b.v[0], acc, 0, 0, 0);
}

// acc += Σ_s A[s] B[s] over 16 register values per lane (the f32 form's 16 k-steps of 32x32x2):
// two bf16 steps of eight values each
template <int NP>
__device__ __forceinline__ void mfma16(f32x16& acc, const float* a, const float* b) {
  if constexpr (NP == 0) {
#pragma unroll
    for (int s = 0; s < 16; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], b[s], acc, 0, 0, 0);
  } else {
#pragma unroll
    for (int m = 0; m < 2; ++m) mfma_x<NP>(acc, planes8<NP>(a + 8 * m), planes8<NP>(b + 8 * m));
  }
}

// row of accumulator register r in lane half h (32x32 C/D layout)
__device__ __forceinline__ int crow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// Orders one wave's LDS writes before its later LDS reads of other lanes' data.  A release
// fence would also wait for every outstanding GLOBAL store of the wave (vmcnt(0)) and stall
// the head loop on its own dY stores; only the LDS counter matters here.
__device__ __forceinline__ void wave_lds_fence() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

}  // namespace
