// bf16 launches with a MN-contiguous A operand (weight gradients).
#include "gemm_split_impl.h"

namespace nrfast {

int launch_split_mn1(const Args& g, int am, int bm, int splits, hipStream_t s) {
  return launch_split_mn<1>(g, am, bm, splits, s);
}

}  // namespace nrfast
