// 64x64-tile instantiations of the exact-f32 fast GEMM (small problems), a translation unit of
// their own so they compile in parallel with the 128x128 ones.
#include "gemm_fast_impl.h"

namespace nrfast {

int launch_modes64(const Args& g, int am, int bm, int splits, hipStream_t s) {
  return launch_modes<64, 64>(g, am, bm, splits, NR_GEMM_F32, s);
}

}  // namespace nrfast
