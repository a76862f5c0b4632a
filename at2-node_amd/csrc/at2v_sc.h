// at2v_sc.h — scalars mod l = 2^252 + 27742317777372353535851937790883648493 (8 x u32, little-endian).
//   sc_is_canonical : V1, s < l (dalek check_scalar / from_canonical_bytes)
//   sc_reduce512    : V3, k = LE512(SHA-512(R||A||M)) mod l (Barrett, HAC 14.42, base 2^32)
//   sc_recode4/8    : signed fixed-window digits for the wavefront-uniform ladder
#pragma once
#include "at2v_fe_base.h"

namespace at2v {

#define AT2V_L_WORDS {0x5cf5d3edu, 0x5812631au, 0xa2f79cd6u, 0x14def9deu, 0u, 0u, 0u, 0x10000000u}

AT2V_HD AT2V_INLINE int sc_is_canonical(const uint32_t s[8]) {
  const uint32_t l[8] = AT2V_L_WORDS;
  // s < l  <=>  borrow out of s - l
  uint64_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint64_t d = (uint64_t)s[i] - l[i] - borrow;
    borrow = (d >> 63) & 1;
  }
  return (int)borrow;
}

// r (9 words) -= l when r >= l
AT2V_HD AT2V_INLINE void sc_cond_sub_l9(uint32_t r[9]) {
  const uint32_t l[8] = AT2V_L_WORDS;
  uint32_t t[9];
  uint64_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    uint64_t d = (uint64_t)r[i] - (i < 8 ? l[i] : 0u) - borrow;
    t[i] = (uint32_t)d;
    borrow = (d >> 63) & 1;
  }
  const int ge = borrow == 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) r[i] = ge ? t[i] : r[i];
}

// k = x mod l for a 512-bit x (16 LE words). Barrett with b = 2^32, k = 8, mu = floor(b^16 / l).
AT2V_HD AT2V_INLINE void sc_reduce512(uint32_t k[8], const uint32_t x[16]) {
  const uint32_t mu[9] = {0x0a2c131bu, 0xed9ce5a3u, 0x086329a7u, 0x2106215du, 0xffffffebu,
                          0xffffffffu, 0xffffffffu, 0xffffffffu, 0x0000000fu};
  const uint32_t l[8] = AT2V_L_WORDS;
  // q1 = floor(x / b^7) : words 7..15 (9 words); q2 = q1 * mu (18 words); q3 = floor(q2 / b^9)
  uint32_t q2[18];
#pragma unroll
  for (int i = 0; i < 18; ++i) q2[i] = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      uint64_t t = (uint64_t)x[7 + i] * mu[j] + q2[i + j] + carry;
      q2[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    q2[i + 9] = (uint32_t)carry;
  }
  // r2 = (q3 * l) mod b^9 ; q3 = q2[9..17]
  uint32_t r2[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) r2[i] = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (i + j < 9) {
        uint64_t t = (uint64_t)q2[9 + i] * l[j] + r2[i + j] + carry;
        r2[i + j] = (uint32_t)t;
        carry = t >> 32;
      }
    }
    if (i + 8 < 9) r2[i + 8] = (uint32_t)carry;  // row 0's carry lands in word 8
  }
  // r = (x mod b^9) - r2  (mod b^9), then at most two subtractions of l
  uint32_t r[9];
  uint64_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    uint64_t d = (uint64_t)x[i] - r2[i] - borrow;
    r[i] = (uint32_t)d;
    borrow = (d >> 63) & 1;
  }
  sc_cond_sub_l9(r);
  sc_cond_sub_l9(r);
#pragma unroll
  for (int i = 0; i < 8; ++i) k[i] = r[i];
}

// Signed radix-16 digits d_0..d_63 of a scalar < 2^253, d_i in [-8, 7] (d_63 in [0, 2]),
// stored as (d_i + 8) nibbles: word j holds digits 8j..8j+7 (digit 8j+m at bits 4m..4m+3).
AT2V_HD AT2V_INLINE void sc_recode4(uint32_t out[8], const uint32_t s[8]) {
  int carry = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    uint32_t w = 0;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      int d = (int)((s[j] >> (4 * m)) & 15) + carry;
      carry = (d + 8) >> 4;
      d -= carry << 4;
      w |= (uint32_t)(d + 8) << (4 * m);
    }
    out[j] = w;
  }
  // carry out of digit 63 is 0 for s < 2^253 (digit 63 <= 1 + 1)
}

// Signed radix-16 digits d_i in [-7, 8] (stored as d_i + 7 nibbles): a value < 2^(4m-1) needs only m digits
// (its top nibble <= 7 plus a carry is at most 8, so nothing carries out). Used for the half-size
// scalars, whose window count is the wave maximum of that m.
AT2V_HD AT2V_INLINE void sc_recode4_hi8(uint32_t out[8], const uint32_t s[8]) {
  int carry = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    uint32_t w = 0;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      int d = (int)((s[j] >> (4 * m)) & 15) + carry;
      carry = (d + 7) >> 4;
      d -= carry << 4;
      w |= (uint32_t)(d + 7) << (4 * m);
    }
    out[j] = w;
  }
}

// Signed radix-256 digits e_0..e_31 of a scalar < 2^253, e_i in [-128, 127], stored as (e_i + 128)
// bytes: word j holds digits 4j..4j+3.
AT2V_HD AT2V_INLINE void sc_recode8(uint32_t out[8], const uint32_t s[8]) {
  int carry = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    uint32_t w = 0;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      int d = (int)((s[j] >> (8 * m)) & 255) + carry;
      carry = (d + 128) >> 8;
      d -= carry << 8;
      w |= (uint32_t)(d + 128) << (8 * m);
    }
    out[j] = w;
  }
}

// Signed radix-2^16 digits e_0..e_15 of a scalar < 2^253, e_i in [-2^15, 2^15), stored as (e_i + 2^15)
// halfwords: word j holds digits 2j (low half) and 2j+1 (high half).
AT2V_HD AT2V_INLINE void sc_recode16(uint32_t out[8], const uint32_t s[8]) {
  int carry = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    uint32_t w = 0;
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      int d = (int)((s[j] >> (16 * m)) & 0xffff) + carry;
      carry = (d + 0x8000) >> 16;
      d -= carry << 16;
      w |= (uint32_t)(d + 0x8000) << (16 * m);
    }
    out[j] = w;
  }
}

// Signed radix-2^WB digits e_0..e_{ND-1} of a scalar < 2^253 (WB in {16, 20, 24}, ND = ceil(254 / WB)),
// e_j in [-2^(WB-1), 2^(WB-1)), stored one per word as e_j + 2^(WB-1).
template <int WB>
struct ScWin {
  static constexpr int ND = (254 + WB - 1) / WB;
};
template <int WB>
AT2V_HD AT2V_INLINE void sc_recode_w(uint32_t out[ScWin<WB>::ND], const uint32_t s[8]) {
  constexpr int ND = ScWin<WB>::ND;
  int carry = 0;
#pragma unroll
  for (int j = 0; j < ND; ++j) {
    const int bit = WB * j, k = bit >> 5, sh = bit & 31;
    uint32_t raw = k < 8 ? (s[k] >> sh) : 0u;
    if (sh && k + 1 < 8) raw |= s[k + 1] << (32 - sh);
    raw &= (1u << WB) - 1u;
    int d = (int)raw + carry;
    carry = (d + (1 << (WB - 1))) >> WB;
    d -= carry << WB;
    out[j] = (uint32_t)(d + (1 << (WB - 1)));
  }
}

}  // namespace at2v
