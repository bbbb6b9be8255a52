// bf16x6 launches with a MN-contiguous A operand (weight gradients).
#include "gemm_split_impl.h"

namespace nrfast {

int launch_split_mn3(const Args& g, int am, int bm, int splits, hipStream_t s) {
  return launch_split_mn<3>(g, am, bm, splits, s);
}

// dispatcher: np = 3 (bf16x6) or 1 (bf16)
int launch_split_modes(const Args& g, int am, int bm, int splits, int np, hipStream_t s) {
  if (is_kc(am)) return np == 1 ? launch_split_kc1(g, am, bm, splits, s) : launch_split_kc3(g, am, bm, splits, s);
  return np == 1 ? launch_split_mn1(g, am, bm, splits, s) : launch_split_mn3(g, am, bm, splits, s);
}

}  // namespace nrfast
