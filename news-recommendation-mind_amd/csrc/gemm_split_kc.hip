// bf16x6 launches with a K-contiguous A operand (projections, dgrads).
#include "gemm_split_impl.h"

namespace nrfast {

int launch_split_kc(const Args& g, int am, int bm, int splits, hipStream_t s) {
  const bool atomic_epi = g.epi == NR_EPI_ATOMIC || g.epi == NR_EPI_SCATTER;
#define NR_SAB(A_, B_, TR_) \
  if (am == A_ && bm == B_ && atomic_epi == !TR_) return launch_split<A_, B_, TR_>(g, splits, s);
  NR_SAB(KC_GATHER, KC_PLAIN, true)
  NR_SAB(KC_CONV3, KC_PLAIN, true)
  NR_SAB(KC_PLAIN, KC_PLAIN, true)
  NR_SAB(KC_PLAIN, MN_PLAIN, true)
  NR_SAB(KC_PLAIN, MN_PLAIN, false)
#undef NR_SAB
  return -1;
}

}  // namespace nrfast
