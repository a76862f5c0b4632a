// at2v_ge.h — twisted Edwards (a = -1) group law over at2v_fe, extended coordinates.
//
// Formulas (Hisil–Wong–Carter–Dawson 2008, complete for a = -1, d non-square; valid for every
// input including the identity and small-order points, which cofactorless verify needs —
// SURVEY Appendix A V4):
//   dbl  p2 -> p1p1 : 3 S + 1 S2 (2Z^2), outputs are k<=3-term sums of carried values
//   add  p3 + cached(Y+X, Y-X, 2Z, 2dT) -> p1p1 : 4 M
//   madd p3 + niels (y+x, y-x, 2dxy), Z2 = 1  -> p1p1 : 3 M
//   p1p1 -> p2 : 3 M,  p1p1 -> p3 : 4 M
// p1p1 (X, Y, Z, T) represents x = X/Z, y = Y/T.
#pragma once
#include "at2v_fe.h"

namespace at2v {

struct ge_p2 { fe X, Y, Z; };
struct ge_p3 { fe X, Y, Z, T; };
struct ge_p1p1 { fe X, Y, Z, T; };
struct ge_cached { fe YpX, YmX, Z2, T2d; };
struct ge_niels { fe ypx, ymx, xy2d; };

AT2V_HD AT2V_INLINE void ge_p3_identity(ge_p3& p) {
  fe_0(p.X);
  fe_1(p.Y);
  fe_1(p.Z);
  fe_0(p.T);
}

AT2V_HD AT2V_INLINE void ge_p1p1_to_p2(ge_p2& r, const ge_p1p1& p) {
  fe_mul(r.X, p.X, p.T);
  fe_mul(r.Y, p.Y, p.Z);
  fe_mul(r.Z, p.Z, p.T);
}

AT2V_HD AT2V_INLINE void ge_p1p1_to_p3(ge_p3& r, const ge_p1p1& p) {
  fe_mul(r.X, p.X, p.T);
  fe_mul(r.Y, p.Y, p.Z);
  fe_mul(r.Z, p.Z, p.T);
  fe_mul(r.T, p.X, p.Y);
}

// dbl-2008-hwcd with the four intermediates negated (E' = -E, F' = -F, G' = -G, H' = -H; the
// products are unchanged) so no subtraction has a 2-term subtrahend:
//   XX = X^2, YY = Y^2, ZZ2 = 2 Z^2, t0 = (X+Y)^2
//   x3 = E'/G',  y3 = H'/F'   with  E' = XX+YY-t0, G' = XX-YY, H' = XX+YY, F' = ZZ2+XX-YY
AT2V_HD AT2V_INLINE void ge_p2_dbl(ge_p1p1& r, const ge_p2& p) {
  fe XX, YY, ZZ2, s, t0;
  fe_sq(XX, p.X);
  fe_sq(YY, p.Y);
  fe_sq2(ZZ2, p.Z);
  fe_add(s, p.X, p.Y);
  fe_sq(t0, s);
  fe_add(r.Y, XX, YY);   // H'   2-term
  fe_sub(r.Z, XX, YY);   // G'   2-term
  fe_sub(r.X, r.Y, t0);  // E'   3-term
  fe_add(r.T, ZZ2, r.Z); // F'   3-term
}

AT2V_HD AT2V_INLINE void ge_p3_to_p2(ge_p2& r, const ge_p3& p) {
  r.X = p.X;
  r.Y = p.Y;
  r.Z = p.Z;
}

AT2V_HD AT2V_INLINE void ge_p3_dbl(ge_p1p1& r, const ge_p3& p) {
  ge_p2 q;
  ge_p3_to_p2(q, p);
  ge_p2_dbl(r, q);
}

// p3 + cached (add-2008-hwcd-3): A = (Y1-X1)(Y2-X2), B = (Y1+X1)(Y2+X2), C = T1*2dT2, D = Z1*2Z2,
// x3 = (B-A)/(D+C), y3 = (B+A)/(D-C)
AT2V_HD AT2V_INLINE void ge_add(ge_p1p1& r, const ge_p3& p, const ge_cached& q) {
  fe a, b, c, d, t;
  fe_sub(t, p.Y, p.X);
  fe_mul(a, t, q.YmX);
  fe_add(t, p.Y, p.X);
  fe_mul(b, t, q.YpX);
  fe_mul(c, p.T, q.T2d);
  fe_mul(d, p.Z, q.Z2);
  fe_sub(r.X, b, a);  // E
  fe_add(r.Y, b, a);  // H
  fe_add(r.Z, d, c);  // G
  fe_sub(r.T, d, c);  // F
}

// p3 + affine Niels point (Z2 = 1)
AT2V_HD AT2V_INLINE void ge_madd(ge_p1p1& r, const ge_p3& p, const ge_niels& q) {
  fe a, b, c, d, t;
  fe_sub(t, p.Y, p.X);
  fe_mul(a, t, q.ymx);
  fe_add(t, p.Y, p.X);
  fe_mul(b, t, q.ypx);
  fe_mul(c, p.T, q.xy2d);
  fe_add(d, p.Z, p.Z);  // 2-term
  fe_sub(r.X, b, a);
  fe_add(r.Y, b, a);
  fe_add(r.Z, d, c);    // 3-term
  fe_sub(r.T, d, c);    // 3-term
}

AT2V_HD AT2V_INLINE void ge_p3_to_cached(ge_cached& r, const ge_p3& p) {
  fe_add(r.YpX, p.Y, p.X);
  fe_carry32(r.YpX);
  fe_sub(r.YmX, p.Y, p.X);
  fe_carry32(r.YmX);
  fe_add(r.Z2, p.Z, p.Z);
  fe_carry32(r.Z2);
  fe_mul(r.T2d, p.T, FE_D2);
}

AT2V_HD AT2V_INLINE void ge_cached_identity(ge_cached& r) {
  fe_1(r.YpX);
  fe_1(r.YmX);
  fe_1(r.Z2);
  r.Z2.v[0] = 2;
  fe_0(r.T2d);
}

// negation of a cached point: (Y+X, Y-X, 2Z, 2dT) -> (Y-X, Y+X, 2Z, -2dT); applied when neg = 1
AT2V_HD AT2V_INLINE void ge_cached_cneg(ge_cached& r, int neg) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const int32_t a = r.YpX.v[i], b = r.YmX.v[i], t = r.T2d.v[i];
    r.YpX.v[i] = neg ? b : a;
    r.YmX.v[i] = neg ? a : b;
    r.T2d.v[i] = neg ? -t : t;
  }
}

AT2V_HD AT2V_INLINE void ge_niels_cneg(ge_niels& r, int neg) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const int32_t a = r.ypx.v[i], b = r.ymx.v[i], t = r.xy2d.v[i];
    r.ypx.v[i] = neg ? b : a;
    r.ymx.v[i] = neg ? a : b;
    r.xy2d.v[i] = neg ? -t : t;
  }
}

// affine Niels form (y+x, y-x, 2dxy) of a p2 point (one inversion), carried limbs
AT2V_HD AT2V_INLINE void ge_p2_to_niels(ge_niels& r, const ge_p2& p) {
  fe zi, x, y;
  fe_invert(zi, p.Z);
  fe_mul(x, p.X, zi);
  fe_mul(y, p.Y, zi);
  fe_add(r.ypx, y, x);
  fe_carry32(r.ypx);
  fe_sub(r.ymx, y, x);
  fe_carry32(r.ymx);
  fe_mul(r.xy2d, x, y);
  fe_mul(r.xy2d, r.xy2d, FE_D2);
}

// enc(P) = canonical y with bit 255 = x & 1 (x = X/Z, y = Y/Z), as 8 LE words
AT2V_HD AT2V_INLINE void ge_p2_tobytes(uint32_t out[8], const ge_p2& p) {
  fe zi, x, y;
  fe_invert(zi, p.Z);
  fe_mul(x, p.X, zi);
  fe_mul(y, p.Y, zi);
  uint32_t xb[8];
  fe_tobytes(out, y);
  fe_tobytes(xb, x);
  out[7] ^= (xb[0] & 1u) << 31;
}

// dalek CompressedEdwardsY::decompress: y = LE255(s) mod p, no canonicity
// check; (ok, x) = sqrt_ratio_i(y^2 - 1, d y^2 + 1); fail if !ok; x = -x if the sign bit is set
// (also when x = 0). Returns 1 on success.
AT2V_HD AT2V_INLINE int ge_frombytes(ge_p3& h, const uint32_t s[8]) {
  fe u, v, v3, vxx, chk, one, t;
  fe_frombytes(h.Y, s);
  fe_1(h.Z);
  fe_1(one);
  fe_sq(u, h.Y);
  fe_mul(v, u, FE_D);
  fe_sub(u, u, one);   // u = y^2 - 1   (2-term)
  fe_add(v, v, one);   // v = d y^2 + 1 (2-term)
  fe_carry32(u);
  fe_carry32(v);
  fe_sq(v3, v);
  fe_mul(v3, v3, v);   // v^3
  fe_sq(t, v3);
  fe_mul(t, t, v);     // v^7
  fe_mul(t, t, u);     // u v^7
  fe_pow22523(t, t);   // (u v^7)^((p-5)/8)
  fe_mul(t, t, v3);
  fe_mul(h.X, t, u);   // r = u v^3 (u v^7)^((p-5)/8)
  fe_sq(vxx, h.X);
  fe_mul(vxx, vxx, v); // v r^2
  fe_sub(chk, vxx, u);
  const int correct = fe_iszero(chk);
  fe_add(chk, vxx, u);
  const int flipped = fe_iszero(chk);
  fe_mul(t, u, FE_SQRTM1);
  fe_add(chk, vxx, t);  // v r^2 == -u*i  <=>  v r^2 + u i == 0
  const int flipped_i = fe_iszero(chk);
  fe_mul(t, h.X, FE_SQRTM1);
  fe_select(h.X, h.X, t, flipped | flipped_i);
  fe_neg(t, h.X);
  fe_select(h.X, h.X, t, fe_isnegative(h.X));  // non-negative root
  fe_neg(t, h.X);
  fe_select(h.X, h.X, t, (int)(s[7] >> 31));   // apply the encoded sign
  fe_mul(h.T, h.X, h.Y);
  return correct | flipped;
}

}  // namespace at2v
