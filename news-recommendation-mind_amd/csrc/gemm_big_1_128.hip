// Large-tile bf16 GEMM instantiations: NP = 1 (bf16), BN = 128 (gemm_big_impl.h).
#include "gemm_big_impl.h"

namespace nrfast {

int launch_big_1_128(const Args& g, int am, int bm, int splits, hipStream_t s) {
  return launch_big_modes<1, 128>(g, am, bm, splits, s);
}

}  // namespace nrfast
