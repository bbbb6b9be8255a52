// Large-tile bf16 GEMM instantiations: NP = 3 (bf16x6), BN = 256 (gemm_big_impl.h).
#include "gemm_big_impl.h"

namespace nrfast {

int launch_big_3_256(const Args& g, int am, int bm, int splits, hipStream_t s) {
  return launch_big_modes<3, 256>(g, am, bm, splits, s);
}

}  // namespace nrfast
