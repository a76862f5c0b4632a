// at2v_gu.h — twisted Edwards (a = -1) group law over the unsigned field at2v_fu.
//
// Same formulas as at2v_ge.h (Hisil–Wong–Carter–Dawson 2008, complete for a = -1, d non-square: valid for every input
// including the identity and small-order points, which cofactorless verify needs — SURVEY Appendix A V4), rearranged
// so every subtraction is a + K - b with K dominating b, and every product's operands stay inside the classes proven
// by tools/gen_fu.py (check_group_law mirrors this file). Conventions:
//   p1p1 (X, Y, Z, T) represents x = X/Z, y = Y/T; X may be "wide" (fu_mul f-side only), Y, Z, T are g-side operands.
//   p1p1 -> p2/p3: X3 = X*T, Y3 = Y*Z (Z*Y with AT2V_GU_SHARE), Z3 = Z*T (, T3 = X*Y) — the first operand is fu_mul's f.
// Products whose inputs keep the top carry below 2^32 (proven per site by check_group_law) use the one-MAD wrap
// variants (fu_mul_n / _wn / _nn, fu_sqc_x2, fu_sq_sq2_n).
#pragma once
#include "at2v_fu.h"

namespace at2v {

// AT2V_GU_X2 = 1: the group law's independent products run as interleaved pairs (two MAD chains in one asm block, round
// 2); 0 (default since round 3): one product at a time through the single-product variants (same columns; a pair's
// one-MAD wraps become the single functions' own wraps, always valid): fewer live registers, +0.4% in two A/B runs
// (profiles/r03r, r03s).
#ifndef AT2V_GU_X2
#define AT2V_GU_X2 0
#endif
#if AT2V_GU_X2
#define GU_MUL_WN(a, f0, g0, b, f1, g1) fu_mul_wn(a, f0, g0, b, f1, g1)
#define GU_MUL_NN(a, f0, g0, b, f1, g1) fu_mul_nn(a, f0, g0, b, f1, g1)
#define GU_MUL_X2(a, f0, g0, b, f1, g1) fu_mul_x2(a, f0, g0, b, f1, g1)
#define GU_SQC_X2(a, f0, b, f1) fu_sqc_x2(a, f0, b, f1)
#define GU_SQ_SQ2_N(a, f0, b, f1) fu_sq_sq2_n(a, f0, b, f1)
#else
#define GU_MUL_WN(a, f0, g0, b, f1, g1) (fu_mul(a, f0, g0), fu_mul_n(b, f1, g1))
#define GU_MUL_NN(a, f0, g0, b, f1, g1) (fu_mul_n(a, f0, g0), fu_mul_n(b, f1, g1))
#define GU_MUL_X2(a, f0, g0, b, f1, g1) (fu_mul(a, f0, g0), fu_mul(b, f1, g1))
#define GU_SQC_X2(a, f0, b, f1) (fu_sqc(a, f0), fu_sqc(b, f1))
#define GU_SQ_SQ2_N(a, f0, b, f1) (fu_sq(a, f0), fu_sq2(b, f1))
#endif

// AT2V_GU_SHARE = 1: Y3 = Z*Y, so the conversion's products use only T and Y as the x19-premultiplied operand and X and
// Z as the doubled-odd-limb operand; the compiler computes each of those once (CSE): 14 fewer VALU ops per p1p1 -> p3,
// 5 per p1p1 -> p2.
#ifndef AT2V_GU_SHARE
#define AT2V_GU_SHARE 1
#endif

struct gu_p2 { fu X, Y, Z; };
struct gu_p3 { fu X, Y, Z, T; };
struct gu_p1p1 { fu X, Y, Z, T; };
struct gu_cached { fu YpX, YmX, Z2, T2d; };
struct gu_niels { fu ypx, ymx, xy2d; };

AT2V_HD AT2V_INLINE void gu_p3_identity(gu_p3& p) {
  fu_0(p.X);
  fu_1(p.Y);
  fu_1(p.Z);
  fu_0(p.T);
}

AT2V_HD AT2V_INLINE void gu_p1p1_to_p2(gu_p2& r, const gu_p1p1& p) {
#if AT2V_GU_SHARE
  GU_MUL_WN(r.X, p.X, p.T, r.Y, p.Z, p.Y);
#else
  GU_MUL_WN(r.X, p.X, p.T, r.Y, p.Y, p.Z);
#endif
  fu_mul(r.Z, p.Z, p.T);
}

AT2V_HD AT2V_INLINE void gu_p1p1_to_p3(gu_p3& r, const gu_p1p1& p) {
#if AT2V_GU_SHARE
  GU_MUL_WN(r.X, p.X, p.T, r.Y, p.Z, p.Y);
#else
  GU_MUL_WN(r.X, p.X, p.T, r.Y, p.Y, p.Z);
#endif
  GU_MUL_X2(r.Z, p.Z, p.T, r.T, p.X, p.Y);
}

// dbl-2008-hwcd, p2 -> p1p1: XX = X^2, YY = Y^2, ZZ2 = 2 Z^2, t0 = (X+Y)^2;
//   X' = XX + YY - t0 (= -2XY), Z' = XX - YY, Y' = XX + YY, T' = ZZ2 + XX - YY (even limbs carried into odd ones)
//   x3 = X'/Z' = 2XY/(Y^2 - X^2), y3 = Y'/T' = (X^2 + Y^2)/(2Z^2 - Y^2 + X^2)
AT2V_HD AT2V_INLINE void gu_p2_dbl(gu_p1p1& r, const gu_p2& p) {
  fu XX, YY, ZZ2, s, t0;
  fu_add(s, p.X, p.Y);
  GU_SQC_X2(XX, p.X, YY, p.Y);
  GU_SQ_SQ2_N(t0, s, ZZ2, p.Z);
  fu_add(r.Y, XX, YY);
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    r.X.v[i] = r.Y.v[i] + FU_KC.v[i] - t0.v[i];
    r.Z.v[i] = XX.v[i] + FU_KC.v[i] - YY.v[i];
    r.T.v[i] = ZZ2.v[i] + r.Z.v[i];
  }
  fu_pcarry_even(r.T);
}

AT2V_HD AT2V_INLINE void gu_p3_to_p2(gu_p2& r, const gu_p3& p) {
  r.X = p.X;
  r.Y = p.Y;
  r.Z = p.Z;
}

// p3 + cached (add-2008-hwcd-3): A = (Y1-X1)(Y2-X2), B = (Y1+X1)(Y2+X2), C = T1*2dT2, D = Z1*2Z2,
// x3 = (B-A)/(D+C), y3 = (B+A)/(D-C)
AT2V_HD AT2V_INLINE void gu_add(gu_p1p1& r, const gu_p3& p, const gu_cached& q) {
  fu a, b, c, d, ym, yp;
  fu_sub(ym, p.Y, p.X, FU_KC);
  fu_add(yp, p.Y, p.X);
  GU_MUL_WN(a, ym, q.YmX, b, yp, q.YpX);
  GU_MUL_NN(c, p.T, q.T2d, d, p.Z, q.Z2);
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    r.X.v[i] = b.v[i] + FU_KC.v[i] - a.v[i];  // E
    r.Y.v[i] = b.v[i] + a.v[i];                // H
    r.Z.v[i] = d.v[i] + c.v[i];                // G
    r.T.v[i] = d.v[i] + FU_KC.v[i] - c.v[i];  // F
  }
}

// p3 + affine Niels point (Z2 = 1)
AT2V_HD AT2V_INLINE void gu_madd(gu_p1p1& r, const gu_p3& p, const gu_niels& q) {
  fu a, b, c, ym, yp;
  fu_sub(ym, p.Y, p.X, FU_KC);
  fu_add(yp, p.Y, p.X);
  GU_MUL_NN(a, ym, q.ymx, b, yp, q.ypx);
  fu_mul_n(c, p.T, q.xy2d);
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint32_t d = p.Z.v[i] + p.Z.v[i];
    r.X.v[i] = b.v[i] + FU_KC.v[i] - a.v[i];  // E
    r.Y.v[i] = b.v[i] + a.v[i];                // H
    r.Z.v[i] = d + c.v[i];                     // G
    r.T.v[i] = d + FU_KC.v[i] - c.v[i];       // F
  }
  fu_pcarry_even(r.T);
}

AT2V_HD AT2V_INLINE void gu_p3_to_cached(gu_cached& r, const gu_p3& p) {
  fu_add(r.YpX, p.Y, p.X);
  fu_sub(r.YmX, p.Y, p.X, FU_KC);
  fu_add(r.Z2, p.Z, p.Z);
  fu_mul_n(r.T2d, p.T, FU_D2);
}

AT2V_HD AT2V_INLINE void gu_cached_identity(gu_cached& r) {
  fu_1(r.YpX);
  fu_1(r.YmX);
  fu_1(r.Z2);
  r.Z2.v[0] = 2;
  fu_0(r.T2d);
}

// negation of a cached point: (Y+X, Y-X, 2Z, 2dT) -> (Y-X, Y+X, 2Z, K - 2dT); applied when neg = 1
AT2V_HD AT2V_INLINE void gu_cached_cneg(gu_cached& r, int neg) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint32_t a = r.YpX.v[i], b = r.YmX.v[i], t = r.T2d.v[i];
    r.YpX.v[i] = neg ? b : a;
    r.YmX.v[i] = neg ? a : b;
    r.T2d.v[i] = neg ? FU_KC.v[i] - t : t;
  }
}

AT2V_HD AT2V_INLINE void gu_niels_cneg(gu_niels& r, int neg) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint32_t a = r.ypx.v[i], b = r.ymx.v[i], t = r.xy2d.v[i];
    r.ypx.v[i] = neg ? b : a;
    r.ymx.v[i] = neg ? a : b;
    r.xy2d.v[i] = neg ? FU_KC.v[i] - t : t;
  }
}

// dalek CompressedEdwardsY::decompress of two encodings at once: y = LE255(s) mod p, no
// canonicity check; (ok, x) = sqrt_ratio_i(y^2 - 1, d y^2 + 1); fail if !ok; x = -x if the sign bit is set (also
// when x = 0). The two exponentiations run as one interleaved pair. Returns the success bits in ok[0], ok[1].
AT2V_HD AT2V_INLINE void gu_frombytes_x2(gu_p3& h0, const uint32_t s0[8], gu_p3& h1, const uint32_t s1[8], int ok[2]) {
  gu_p3* hs[2] = {&h0, &h1};
  const uint32_t* ss[2] = {s0, s1};
  fu u[2], v[2], v3[2], t[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    gu_p3& h = *hs[k];
    fu_frombytes(h.Y, ss[k]);
    fu_1(h.Z);
  }
  fu_sqc_x2(u[0], h0.Y, u[1], h1.Y);
  fu_mulc_x2(v[0], u[0], FU_D, v[1], u[1], FU_D);
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    fu_add(u[k], u[k], FU_PM1);  // u = y^2 - 1  (y^2 + p - 1)
    v[k].v[0] += 1;              // v = d y^2 + 1
  }
  fu_sq_x2(v3[0], v[0], v3[1], v[1]);
  fu_mul_x2(v3[0], v3[0], v[0], v3[1], v3[1], v[1]);   // v^3
  fu_sqc_x2(t[0], v3[0], t[1], v3[1]);
  fu_mul_x2(t[0], t[0], v[0], t[1], t[1], v[1]);       // v^7
  fu_mul_x2(t[0], u[0], t[0], t[1], u[1], t[1]);       // u v^7
  fu_pow22523_x2(t[0], t[0], t[1], t[1]);              // (u v^7)^((p-5)/8)
  fu_mulc_x2(t[0], t[0], v3[0], t[1], t[1], v3[1]);
  fu_mul_x2(h0.X, u[0], t[0], h1.X, u[1], t[1]);       // r = u v^3 (u v^7)^((p-5)/8)
  fu vxx[2];
  fu_sqc_x2(vxx[0], h0.X, vxx[1], h1.X);
  fu_mul_x2(vxx[0], v[0], vxx[0], vxx[1], v[1], vxx[1]);  // v r^2
  fu ui[2], xi[2];
  fu_mul_x2(ui[0], u[0], FU_SQRTM1, ui[1], u[1], FU_SQRTM1);
  fu_mulc_x2(xi[0], h0.X, FU_SQRTM1, xi[1], h1.X, FU_SQRTM1);
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    gu_p3& h = *hs[k];
    fu chk;
    fu_sub(chk, vxx[k], u[k], FU_K2C);
    const int correct = fu_iszero(chk);
    fu_add(chk, vxx[k], u[k]);
    const int flipped = fu_iszero(chk);
    fu_add(chk, vxx[k], ui[k]);  // v r^2 == -u*i  <=>  v r^2 + u i == 0
    const int flipped_i = fu_iszero(chk);
    fu_select(h.X, h.X, xi[k], flipped | flipped_i);
    fu neg;
    fu_neg(neg, h.X, FU_KC);
    fu_select(h.X, h.X, neg, fu_isnegative(h.X));  // non-negative root
    fu_neg(neg, h.X, FU_KC);
    fu_select(h.X, h.X, neg, (int)(ss[k][7] >> 31));  // apply the encoded sign
    fu_carry(h.X);
    ok[k] = correct | flipped;
  }
  fu_mulc_x2(h0.T, h0.X, h0.Y, h1.T, h1.X, h1.Y);
}

// one encoding (the low-latency kernel decodes A and R on two lanes, one each): same steps as gu_frombytes_x2
AT2V_HD AT2V_INLINE int gu_frombytes(gu_p3& h, const uint32_t s[8]) {
  fu u, v, v3, t;
  fu_frombytes(h.Y, s);
  fu_1(h.Z);
  fu_sqc(u, h.Y);
  fu_mulc(v, u, FU_D);
  fu_add(u, u, FU_PM1);  // u = y^2 - 1
  v.v[0] += 1;           // v = d y^2 + 1
  fu_sq(v3, v);
  fu_mul(v3, v3, v);     // v^3
  fu_sqc(t, v3);
  fu_mul(t, t, v);       // v^7
  fu_mul(t, u, t);       // u v^7
  fu_pow22523(t, t);     // (u v^7)^((p-5)/8)
  fu_mulc(t, t, v3);
  fu_mul(h.X, u, t);     // r = u v^3 (u v^7)^((p-5)/8)
  fu vxx, ui, xi, chk;
  fu_sqc(vxx, h.X);
  fu_mul(vxx, v, vxx);   // v r^2
  fu_mul(ui, u, FU_SQRTM1);
  fu_mulc(xi, h.X, FU_SQRTM1);
  fu_sub(chk, vxx, u, FU_K2C);
  const int correct = fu_iszero(chk);
  fu_add(chk, vxx, u);
  const int flipped = fu_iszero(chk);
  fu_add(chk, vxx, ui);  // v r^2 == -u*i  <=>  v r^2 + u i == 0
  const int flipped_i = fu_iszero(chk);
  fu_select(h.X, h.X, xi, flipped | flipped_i);
  fu neg;
  fu_neg(neg, h.X, FU_KC);
  fu_select(h.X, h.X, neg, fu_isnegative(h.X));  // non-negative root
  fu_neg(neg, h.X, FU_KC);
  fu_select(h.X, h.X, neg, (int)(s[7] >> 31));   // apply the encoded sign
  fu_carry(h.X);
  fu_mulc(h.T, h.X, h.Y);
  return correct | flipped;
}

}  // namespace at2v
