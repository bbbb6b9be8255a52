// Internal: fast-path entry of nr_gemm_f32 (not part of the C ABI).
#pragma once
#include <stdint.h>
#include "../../include/newsrec_hip.h"

// -1: operands not eligible for the fast kernel (caller falls back to the generic one).
int nr_gemm_fast(int64_t M, int64_t N, int64_t K, const nr_operand* A, const nr_operand* B, float* C,
                 int64_t ldc, const float* bias, int32_t epilogue, const nr_operand* c_rows, int64_t pad_row,
                 int32_t split_k, int bm, int bn, const int32_t* m_dev, const int32_t* k_dev,
                 int32_t prec, int32_t max_cus, float* work, int64_t work_elems, float* colsum,
                 int32_t* colsum_folded, hipStream_t stream);
