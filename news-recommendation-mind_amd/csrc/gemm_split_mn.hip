// bf16x6 launches with an MN-contiguous A operand (weight gradients), and the dispatcher.
#include "gemm_split_impl.h"

namespace nrfast {

int launch_split_kc(const Args& g, int am, int bm, int splits, hipStream_t s);   // gemm_split_kc.hip

int launch_split_modes(const Args& g, int am, int bm, int splits, hipStream_t s) {
  if (is_kc(am)) return launch_split_kc(g, am, bm, splits, s);
  const bool atomic_epi = g.epi == NR_EPI_ATOMIC || g.epi == NR_EPI_SCATTER;
  if (!atomic_epi || am != MN_PLAIN) return -1;
  if (bm == MN_GATHER) return launch_split<MN_PLAIN, MN_GATHER, false>(g, splits, s);
  if (bm == MN_PLAIN) return launch_split<MN_PLAIN, MN_PLAIN, false>(g, splits, s);
  if (bm == MN_CONV3 && g.B.seg % 128 == 0) return launch_split<MN_PLAIN, MN_CONV3, false>(g, splits, s);
  return -1;
}

}  // namespace nrfast
