// at2v_fe_fu.h — conversion from the balanced signed field (at2v_fe) to the unsigned one (at2v_fu): the fixed-base
// tables are built by the signed group law (build_btab_kernel, shared with the signer) and consumed by the unsigned
// verify (at2v_verify_fu.h).
#pragma once
#include "at2v_ge.h"
#include "at2v_gu.h"

namespace at2v {

// carried balanced limbs (|v_i| <= 2^(W[i]-1) + 2^16) -> carried unsigned limbs: add 2p limb-wise, then carry
AT2V_HD AT2V_INLINE void fe_to_fu(fu& r, const fe& f) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const int32_t p2 = i == 0 ? (1 << 27) - 38 : (i & 1) ? (1 << 26) - 2 : (1 << 27) - 2;
    r.v[i] = (uint32_t)(f.v[i] + p2);
  }
  fu_carry(r);
}

AT2V_HD AT2V_INLINE void niels_fe_to_fu(gu_niels& r, const ge_niels& n) {
  fe_to_fu(r.ypx, n.ypx);
  fe_to_fu(r.ymx, n.ymx);
  fe_to_fu(r.xy2d, n.xy2d);
}

}  // namespace at2v
