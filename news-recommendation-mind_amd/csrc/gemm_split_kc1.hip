// bf16 launches with a K-contiguous A operand (projections, dgrads).
#include "gemm_split_impl.h"

namespace nrfast {

int launch_split_kc1(const Args& g, int am, int bm, int splits, hipStream_t s) {
  return launch_split_kc<1>(g, am, bm, splits, s);
}

}  // namespace nrfast
