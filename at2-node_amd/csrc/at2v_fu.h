// at2v_fu.h — field layer over unsigned limbs: generated mul/sq (at2v_fu_gen.h), limb-wise
// add/sub with the multiple-of-p constants, carries, (de)serialisation, exponentiation chains (one and two at a
// time) and predicates. Input/output classes of every function are the ones tools/gen_fu.py proves:
//   carried : limb i < 2^W[i] (limb 1 <= 2^25 - 1 + kFuLimb1Spill) — output of every product, fu_carry, fu_frombytes
//   fu_mul f: <= 4 carried units on even limbs, 4.5 on odd ones (limb 9: 6); fu_mul g, fu_sq: <= 3 on even limbs
#pragma once
#include "at2v_fu_gen.h"

namespace at2v {

AT2V_HD AT2V_INLINE void fu_0(fu& h) {
#pragma unroll
  for (int i = 0; i < 10; ++i) h.v[i] = 0;
}
AT2V_HD AT2V_INLINE void fu_1(fu& h) {
  fu_0(h);
  h.v[0] = 1;
}
AT2V_HD AT2V_INLINE void fu_add(fu& h, const fu& f, const fu& g) {
#pragma unroll
  for (int i = 0; i < 10; ++i) h.v[i] = f.v[i] + g.v[i];
}
// h = f + K - g   (K a multiple of p whose limbs dominate g's)
AT2V_HD AT2V_INLINE void fu_sub(fu& h, const fu& f, const fu& g, const fu& K) {
#pragma unroll
  for (int i = 0; i < 10; ++i) h.v[i] = f.v[i] + K.v[i] - g.v[i];
}
// h = K - f
AT2V_HD AT2V_INLINE void fu_neg(fu& h, const fu& f, const fu& K) {
#pragma unroll
  for (int i = 0; i < 10; ++i) h.v[i] = K.v[i] - f.v[i];
}
// h = b ? g : f   (b is 0/1, per lane)
AT2V_HD AT2V_INLINE void fu_select(fu& h, const fu& f, const fu& g, int b) {
#pragma unroll
  for (int i = 0; i < 10; ++i) h.v[i] = b ? g.v[i] : f.v[i];
}

// Floor carry of an element with limbs < 2^32 - 2^12: the result is carried (the second carry into limb 1 is <= 1).
AT2V_HD AT2V_INLINE void fu_carry(fu& h) {
  uint32_t c;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int w = (i & 1) ? 25 : 26;
    c = h.v[i] >> w;
    h.v[i] &= (1u << w) - 1;
    h.v[i + 1] += c;
  }
  c = h.v[9] >> 25;
  h.v[9] &= (1u << 25) - 1;
  h.v[0] += 19 * c;
  c = h.v[0] >> 26;
  h.v[0] &= (1u << 26) - 1;
  h.v[1] += c;
}

// Even limbs carried into the next (odd) limb: even limbs < 2^26, odd limbs grow by < 2^6. Brings a sum of up to four
// carried units under the x19 operand bound of fu_mul's g (tools/gen_fu.py pcarry_even).
AT2V_HD AT2V_INLINE void fu_pcarry_even(fu& h) {
#pragma unroll
  for (int i = 0; i < 10; i += 2) {
    h.v[i + 1] += h.v[i] >> 26;
    h.v[i] &= (1u << 26) - 1;
  }
}

// 32 little-endian bytes (8 LE words) -> carried element. Bit 255 is ignored; values >= p are NOT reduced (dalek
// FieldElement::from_bytes semantics).
AT2V_HD AT2V_INLINE void fu_frombytes(fu& h, const uint32_t w[8]) {
  auto bits = [&](int off, int width) -> uint32_t {
    const int k = off >> 5, s = off & 31;
    const uint64_t v = (uint64_t)w[k] | ((k + 1 < 8) ? ((uint64_t)w[k + 1] << 32) : 0);
    return (uint32_t)((v >> s) & ((1u << width) - 1));
  };
  h.v[0] = bits(0, 26);
  h.v[1] = bits(26, 25);
  h.v[2] = bits(51, 26);
  h.v[3] = bits(77, 25);
  h.v[4] = bits(102, 26);
  h.v[5] = bits(128, 25);
  h.v[6] = bits(153, 26);
  h.v[7] = bits(179, 25);
  h.v[8] = bits(204, 26);
  h.v[9] = bits(230, 25);
}

// Canonical encoding (fully reduced mod p) as 8 little-endian words; any limbs < 2^32 - 2^12.
AT2V_HD AT2V_INLINE void fu_tobytes(uint32_t out[8], const fu& f) {
  uint32_t t[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) t[i] = f.v[i];
#pragma unroll
  for (int pass = 0; pass < 3; ++pass) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      const int w = (i & 1) ? 25 : 26;
      const uint32_t c = t[i] >> w;
      t[i] &= (1u << w) - 1;
      if (i < 9) t[i + 1] += c;
      else t[0] += 19 * c;
    }
  }
  // 0 <= value < 2^255 + 19 with limbs in range; subtract p once if value >= p (value + 19 >= 2^255)
  uint32_t q = (t[0] + 19) >> 26;
#pragma unroll
  for (int i = 1; i < 10; ++i) q = (t[i] + q) >> ((i & 1) ? 25 : 26);
  t[0] += 19 * q;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int w = (i & 1) ? 25 : 26;
    const uint32_t c = t[i] >> w;
    t[i] &= (1u << w) - 1;
    t[i + 1] += c;
  }
  t[9] &= (1u << 25) - 1;
  uint64_t acc = 0;
  int nb = 0, wi = 0;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const int w = (i & 1) ? 25 : 26;
    acc |= (uint64_t)t[i] << nb;
    nb += w;
    while (nb >= 32) {
      out[wi++] = (uint32_t)acc;
      acc >>= 32;
      nb -= 32;
    }
  }
  out[wi] = (uint32_t)acc;  // wi == 7, nb == 31
}

AT2V_HD AT2V_INLINE int fu_iszero(const fu& f) {
  uint32_t b[8];
  fu_tobytes(b, f);
  return (b[0] | b[1] | b[2] | b[3] | b[4] | b[5] | b[6] | b[7]) == 0;
}

AT2V_HD AT2V_INLINE int fu_isnegative(const fu& f) {
  uint32_t b[8];
  fu_tobytes(b, f);
  return (int)(b[0] & 1);
}

// ------------------------------------------------------------------ exponentiation (carried inputs)

// Squaring chains, loops kept rolled. AT2V_SQN_PINGPONG: the loop body squares twice, into a second register set and
// back, so no iteration ends with copying the square over its input (the in-place form costs ~10 v_mov per square).
#ifndef AT2V_SQN_PINGPONG
#define AT2V_SQN_PINGPONG 1
#endif
AT2V_HD AT2V_INLINE void fu_sqn(fu& h, const fu& f, int n) {  // h = f^(2^n), n >= 1
  fu_sqc(h, f);
#if AT2V_SQN_PINGPONG
  int i = 1;
  for (; i + 1 < n; i += 2) {
    fu t;
    fu_sqc(t, h);
    fu_sqc(h, t);
  }
  if (i < n) fu_sqc(h, h);
#else
  for (int i = 1; i < n; ++i) fu_sqc(h, h);
#endif
}
AT2V_HD AT2V_INLINE void fu_sqn_x2(fu& h0, const fu& f0, fu& h1, const fu& f1, int n) {
  fu_sqc_x2(h0, f0, h1, f1);
#if AT2V_SQN_PINGPONG
  int i = 1;
  for (; i + 1 < n; i += 2) {
    fu t0, t1;
    fu_sqc_x2(t0, h0, t1, h1);
    fu_sqc_x2(h0, t0, h1, t1);
  }
  if (i < n) fu_sqc_x2(h0, h0, h1, h1);
#else
  for (int i = 1; i < n; ++i) fu_sqc_x2(h0, h0, h1, h1);
#endif
}

// z250 = z^(2^250 - 1), z11 = z^11 (shared prefix of invert and pow22523)
AT2V_HD AT2V_INLINE void fu_pow250(fu& z250, fu& z11, const fu& z) {
  fu z2, z9, a, b, t;
  fu_sqc(z2, z);            // 2
  fu_sqn(t, z2, 2);         // 8
  fu_mulc(z9, t, z);        // 9
  fu_mulc(z11, z9, z2);     // 11
  fu_sqc(t, z11);           // 22
  fu_mulc(a, t, z9);        // 2^5 - 1
  fu_sqn(t, a, 5);
  fu_mulc(b, t, a);         // 2^10 - 1
  fu_sqn(t, b, 10);
  fu_mulc(a, t, b);         // 2^20 - 1
  fu_sqn(t, a, 20);
  fu_mulc(a, t, a);         // 2^40 - 1
  fu_sqn(t, a, 10);
  fu_mulc(a, t, b);         // 2^50 - 1
  fu_sqn(t, a, 50);
  fu_mulc(b, t, a);         // 2^100 - 1
  fu_sqn(t, b, 100);
  fu_mulc(b, t, b);         // 2^200 - 1
  fu_sqn(t, b, 50);
  fu_mulc(z250, t, a);      // 2^250 - 1
}

AT2V_HD AT2V_INLINE void fu_invert(fu& h, const fu& z) {  // z^(p-2) = z^(2^255 - 21)
  fu z250, z11, t;
  fu_pow250(z250, z11, z);
  fu_sqn(t, z250, 5);
  fu_mulc(h, t, z11);
}

AT2V_HD AT2V_INLINE void fu_pow22523(fu& h, const fu& z) {  // z^((p-5)/8) = z^(2^252 - 3)
  fu z250, z11, t;
  fu_pow250(z250, z11, z);
  fu_sqn(t, z250, 2);
  fu_mulc(h, t, z);
}

// two independent exponentiations with interleaved MAD chains (the A and R decodes of one signature)
AT2V_HD AT2V_INLINE void fu_pow22523_x2(fu& h0, const fu& z0, fu& h1, const fu& z1) {
  fu p2, q2, p9, q9, p11, q11, pa, qa, pb, qb, pt, qt;
  fu_sqc_x2(p2, z0, q2, z1);
  fu_sqn_x2(pt, p2, qt, q2, 2);
  fu_mulc_x2(p9, pt, z0, q9, qt, z1);
  fu_mulc_x2(p11, p9, p2, q11, q9, q2);
  fu_sqc_x2(pt, p11, qt, q11);
  fu_mulc_x2(pa, pt, p9, qa, qt, q9);      // 2^5 - 1
  fu_sqn_x2(pt, pa, qt, qa, 5);
  fu_mulc_x2(pb, pt, pa, qb, qt, qa);      // 2^10 - 1
  fu_sqn_x2(pt, pb, qt, qb, 10);
  fu_mulc_x2(pa, pt, pb, qa, qt, qb);      // 2^20 - 1
  fu_sqn_x2(pt, pa, qt, qa, 20);
  fu_mulc_x2(pa, pt, pa, qa, qt, qa);      // 2^40 - 1
  fu_sqn_x2(pt, pa, qt, qa, 10);
  fu_mulc_x2(pa, pt, pb, qa, qt, qb);      // 2^50 - 1
  fu_sqn_x2(pt, pa, qt, qa, 50);
  fu_mulc_x2(pb, pt, pa, qb, qt, qa);      // 2^100 - 1
  fu_sqn_x2(pt, pb, qt, qb, 100);
  fu_mulc_x2(pb, pt, pb, qb, qt, qb);      // 2^200 - 1
  fu_sqn_x2(pt, pb, qt, qb, 50);
  fu_mulc_x2(pa, pt, pa, qa, qt, qa);      // 2^250 - 1
  fu_sqn_x2(pt, pa, qt, qa, 2);
  fu_mulc_x2(h0, pt, z0, h1, qt, z1);      // 2^252 - 3
}

}  // namespace at2v
