// at2v_fe.h — field layer: generated mul/sq (at2v_fe_gen.h) + exponentiation chains + predicates.
#pragma once
#include "at2v_fe_gen.h"

namespace at2v {

// h = f^(2^n), n >= 1; loop kept rolled (n up to 100) to bound code size
AT2V_HD AT2V_INLINE void fe_sqn(fe& h, const fe& f, int n) {
  fe_sq(h, f);
  for (int i = 1; i < n; ++i) fe_sq(h, h);
}

// z250 = z^(2^250 - 1), z11 = z^11 (shared prefix of invert and pow22523)
AT2V_HD AT2V_INLINE void fe_pow250(fe& z250, fe& z11, const fe& z) {
  fe z2, z9, a, b, t;
  fe_sq(z2, z);             // 2
  fe_sqn(t, z2, 2);         // 8
  fe_mul(z9, t, z);         // 9
  fe_mul(z11, z9, z2);      // 11
  fe_sq(t, z11);            // 22
  fe_mul(a, t, z9);         // 2^5 - 1
  fe_sqn(t, a, 5);
  fe_mul(b, t, a);          // 2^10 - 1
  fe_sqn(t, b, 10);
  fe_mul(a, t, b);          // 2^20 - 1
  fe_sqn(t, a, 20);
  fe_mul(a, t, a);          // 2^40 - 1
  fe_sqn(t, a, 10);
  fe_mul(a, t, b);          // 2^50 - 1
  fe_sqn(t, a, 50);
  fe_mul(b, t, a);          // 2^100 - 1
  fe_sqn(t, b, 100);
  fe_mul(b, t, b);          // 2^200 - 1
  fe_sqn(t, b, 50);
  fe_mul(z250, t, a);       // 2^250 - 1
}

AT2V_HD AT2V_INLINE void fe_invert(fe& h, const fe& z) {  // z^(p-2) = z^(2^255 - 21)
  fe z250, z11, t;
  fe_pow250(z250, z11, z);
  fe_sqn(t, z250, 5);
  fe_mul(h, t, z11);
}

AT2V_HD AT2V_INLINE void fe_pow22523(fe& h, const fe& z) {  // z^((p-5)/8) = z^(2^252 - 3)
  fe z250, z11, t;
  fe_pow250(z250, z11, z);
  fe_sqn(t, z250, 2);
  fe_mul(h, t, z);
}

AT2V_HD AT2V_INLINE int fe_iszero(const fe& f) {
  uint32_t b[8];
  fe_tobytes(b, f);
  return (b[0] | b[1] | b[2] | b[3] | b[4] | b[5] | b[6] | b[7]) == 0;
}

AT2V_HD AT2V_INLINE int fe_isnegative(const fe& f) {
  uint32_t b[8];
  fe_tobytes(b, f);
  return (int)(b[0] & 1);
}

}  // namespace at2v
