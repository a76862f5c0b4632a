// at2v_lattice.h — per-lane 2-dimensional lattice reduction for the half-size verification equation
// (prototype and proof sketch in tools/halfscalar_proto.py).
//
// Given k < l, find (c0, c1) with c0 = c1 * k (mod 8l), c1 odd, both about sqrt(8l) ~ 2^127.5, by
// Euclid's algorithm on (8l, k) stopped at the first remainder below ceil(sqrt(8l)) (Gauss/Lagrange
// reduction in dimension 2; T. Pornin 2020 for the EdDSA use). Modulus 8l instead of l is what keeps the
// verification exactly cofactorless: every curve point has [8l]P = 0, so [c1 k]A = [c0]A for ANY A,
// small-order and mixed-order keys included.
//
// Euclid state: consecutive remainders r_{i-1} >= r_i with cofactors t_i (r_i = t_i * k mod 8l). The
// cofactors alternate in sign, so only their magnitudes m_i are kept: m_{i+1} = m_{i-1} + q * m_i, and
// sign(t_i) = (-1)^(i+1). Quotients come from a double-precision estimate corrected exactly; a quotient
// >= 2^32 (probability ~2^-32 per step) is taken in 32-bit slices.
#pragma once
#include "at2v_sc.h"

namespace at2v {

// 8l = 2^255 + 8 * 27742317777372353535851937790883648493
#define AT2V_8L_WORDS {0xe7ae9f68u, 0xc09318d2u, 0x17bce6b2u, 0xa6f7cef5u, 0u, 0u, 0u, 0x80000000u}
// ceil(sqrt(8l))
#define AT2V_SQRT8L_WORDS {0x754abea0u, 0x597d89b3u, 0xf9de6484u, 0xb504f333u, 0u, 0u, 0u, 0u}

struct U256 {
  uint32_t w[8];
};

AT2V_HD AT2V_INLINE void u256_set(U256& a, const uint32_t v[8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i) a.w[i] = v[i];
}

// a >= b
AT2V_HD AT2V_INLINE bool u256_ge(const U256& a, const U256& b) {
  uint64_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) borrow = (((uint64_t)a.w[i] - b.w[i] - borrow) >> 63) & 1;
  return borrow == 0;
}

// a -= b, returns borrow
AT2V_HD AT2V_INLINE uint32_t u256_sub(U256& a, const U256& b) {
  uint64_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint64_t d = (uint64_t)a.w[i] - b.w[i] - borrow;
    a.w[i] = (uint32_t)d;
    borrow = (d >> 63) & 1;
  }
  return (uint32_t)borrow;
}

// a += b, returns carry
AT2V_HD AT2V_INLINE uint32_t u256_add(U256& a, const U256& b) {
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    c += (uint64_t)a.w[i] + b.w[i];
    a.w[i] = (uint32_t)c;
    c >>= 32;
  }
  return (uint32_t)c;
}

// a -= q * b, returns the borrow word (0 if no underflow)
AT2V_HD AT2V_INLINE uint32_t u256_submul(U256& a, const U256& b, uint32_t q) {
  uint64_t carry = 0;  // q * b running high part
  uint64_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint64_t p = (uint64_t)q * b.w[i] + carry;
    carry = p >> 32;
    const uint64_t d = (uint64_t)a.w[i] - (uint32_t)p - borrow;
    a.w[i] = (uint32_t)d;
    borrow = (d >> 63) & 1;
  }
  return (uint32_t)(carry + borrow);
}

// a += q * b (cofactor magnitudes stay below 8l: no overflow)
AT2V_HD AT2V_INLINE void u256_addmul(U256& a, const U256& b, uint32_t q) {
  uint64_t carry = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint64_t p = (uint64_t)q * b.w[i] + carry + a.w[i];
    a.w[i] = (uint32_t)p;
    carry = p >> 32;
  }
}

// r = b << 32 ws (ws in 1..7, per lane): select network, no dynamically indexed registers
AT2V_HD AT2V_INLINE void u256_shl_words(U256& r, const U256& b, int ws) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint32_t v = 0;
#pragma unroll
    for (int s = 1; s < 8; ++s)
      if (i - s >= 0) v = (ws == s) ? b.w[i - s] : v;
    r.w[i] = v;
  }
}

AT2V_HD AT2V_INLINE double u256_to_double(const U256& a) {
  double v = (double)a.w[7];
#pragma unroll
  for (int i = 6; i >= 0; --i) v = v * 4294967296.0 + (double)a.w[i];
  return v;
}

AT2V_HD AT2V_INLINE int u256_bitlen(const U256& a) {
  int b = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i)
    if (a.w[i]) b = 32 * i + 32 - __builtin_clz(a.w[i]);
  return b;
}

AT2V_HD AT2V_INLINE int imax(int a, int b) { return a > b ? a : b; }

// a := a mod b (a, b > 0), and ma += q * mb for the quotient q = floor(a / b)
AT2V_HD AT2V_INLINE void euclid_reduce(U256& a, U256& ma, const U256& b, const U256& mb) {
  for (int guard = 0; guard < 64 && u256_ge(a, b); ++guard) {
    const double ratio = u256_to_double(a) / u256_to_double(b);
    if (ratio < 4294967296.0) {
      // |estimate - a/b| < 2^-17: the floor is exact or one too large (fixed up here) or one too
      // small (the next pass subtracts one more b)
      uint32_t q = ratio >= 1.0 ? (uint32_t)ratio : 1u;
      if (u256_submul(a, b, q)) {
        u256_add(a, b);
        if (--q == 0) continue;
      }
      u256_addmul(ma, mb, q);
    } else {  // quotient >= 2^32 (rare): subtract an under-estimated 32-bit slice of it, word-shifted
      int ws = 1;
      double r = ratio / 4294967296.0;
      while (r >= 4294967296.0 && ws < 7) {
        r /= 4294967296.0;
        ++ws;
      }
      const uint32_t q = r >= 2.0 ? (uint32_t)(r - 1.0) : 1u;
      U256 bs, mbs;
      u256_shl_words(bs, b, ws);
      u256_shl_words(mbs, mb, ws);
      u256_submul(a, bs, q);  // q * (b << 32 ws) <= a by construction
      u256_addmul(ma, mbs, q);
    }
  }
}

#ifndef AT2V_LEHMER_IEEE_DIV
#define AT2V_LEHMER_IEEE_DIV 0  // 1: IEEE float division in the Lehmer quotient estimate (A/B)
#endif

#ifndef AT2V_LATTICE_PINGPONG
#define AT2V_LATTICE_PINGPONG 1  // two alternating state sets in the reduction loop (0: one set, state copied back)
#endif

#ifndef AT2V_LATTICE_EXACT_MATRIX
#define AT2V_LATTICE_EXACT_MATRIX 1  // exact Euclid steps through lehmer_apply (0: the separate subtract-and-swap path)
#endif

#ifndef AT2V_LATTICE_LEHMER
#define AT2V_LATTICE_LEHMER 2  // 0: plain Euclid, 1: Lehmer on 62-bit leading parts, 2: on 30-bit parts
#endif

// word j of a (0 for j >= 8), j per lane: select network
AT2V_HD AT2V_INLINE uint32_t u256_word(const U256& a, int j) {
  uint32_t v = 0;
#pragma unroll
  for (int s = 0; s < 8; ++s) v = (j == s) ? a.w[s] : v;
  return v;
}

// floor(a / 2^h) mod 2^64 for 0 <= h < 256
AT2V_HD AT2V_INLINE uint64_t u256_shr64(const U256& a, int h) {
  const int wi = h >> 5, sh = h & 31;
  const uint32_t w0 = u256_word(a, wi), w1 = u256_word(a, wi + 1), w2 = u256_word(a, wi + 2);
  const uint32_t lo = sh ? (w0 >> sh) | (w1 << (32 - sh)) : w0;
  const uint32_t hi = sh ? (w1 >> sh) | (w2 << (32 - sh)) : w1;
  return ((uint64_t)hi << 32) | lo;
}

AT2V_HD AT2V_INLINE int64_t iabs64(int64_t v) { return v < 0 ? -v : v; }

// One Lehmer round (Knuth TAOCP 4.5.2 Algorithm L) on u = ra, v = rb: Euclid on the 62-bit leading parts
// x, y with the cofactor matrix (A B; C D), taking a step only while Knuth's two-quotient test proves the
// quotient equals the true one, and while the true v is provably >= the stopping threshold thr (the
// true v / 2^h lies between y + C and y + D). Cofactors stay below 2^31.
AT2V_HD AT2V_INLINE void lehmer_round(int& steps, int64_t& A, int64_t& B, int64_t& Cc, int64_t& D, const U256& ra,
                                      const U256& rb, const U256& thr) {
  const int h = imax(0, u256_bitlen(ra) - 62);
  int64_t x = (int64_t)u256_shr64(ra, h), y = (int64_t)u256_shr64(rb, h);
  const int64_t chat = h < 128 ? (int64_t)(u256_shr64(thr, h) & 0x3fffffffffffffffull) : 0;
  A = 1;
  B = 0;
  Cc = 0;
  D = 1;
  steps = 0;
  for (int it = 0; it < 48; ++it) {
    const int64_t yc = y + Cc, yd = y + D;
    if (yc <= 0 || yd <= 0) break;
    if ((yc < yd ? yc : yd) <= chat) break;  // true v might be < thr: stop before stepping past it
    const int64_t xa = x + A, xb = x + B;
    int64_t q = (int64_t)((double)xa / (double)yc);
    if (q < 0 || q >= (1ll << 30)) break;
    int64_t r = xa - q * yc;  // exact floor(xa / yc): the estimate is within one
    if (r < 0) {
      --q;
      r += yc;
    } else if (r >= yc) {
      ++q;
      r -= yc;
    }
    const int64_t r2 = xb - q * yd;  // Knuth L2: q must also be floor(xb / yd)
    if (r2 < 0 || r2 >= yd) break;
    const int64_t nC = A - q * Cc, nD = B - q * D;
    if (iabs64(nC) >= (1ll << 31) || iabs64(nD) >= (1ll << 31)) break;
    A = Cc;
    Cc = nC;
    B = D;
    D = nD;
    const int64_t ny = x - q * y;
    x = y;
    y = ny;
    ++steps;
  }
}

// Same round on 30-bit leading parts with cofactors below 2^15: every inner-loop operation is a full-rate
// 32-bit VALU op (plus one f32 reciprocal), at the price of ~15 bits per round instead of ~31.
AT2V_HD AT2V_INLINE void lehmer_round32(int& steps, int64_t& A64, int64_t& B64, int64_t& C64, int64_t& D64,
                                        const U256& ra, const U256& rb, const U256& thr) {
  const int h = imax(0, u256_bitlen(ra) - 30);
  const int wi = h >> 5, sh = h & 31;
  auto lead = [&](const U256& a) -> int32_t {
    const uint32_t w0 = u256_word(a, wi), w1 = u256_word(a, wi + 1);
    return (int32_t)((sh ? (w0 >> sh) | (w1 << (32 - sh)) : w0) & 0x3fffffffu);
  };
  int32_t x = lead(ra), y = lead(rb);
  const int32_t chat = h < 128 ? lead(thr) : 0;  // h >= 98 while rb >= thr: thr >> h < 2^30
  int32_t A = 1, B = 0, Cc = 0, D = 1;
  steps = 0;
  for (int it = 0; it < 24; ++it) {
    const int32_t yc = y + Cc, yd = y + D;
    if (yc <= 0 || yd <= 0) break;
    if ((yc < yd ? yc : yd) <= chat) break;  // true v might be < thr
    const int32_t xa = x + A, xb = x + B;
    // xa < 2^31, 1 <= yc, and only q < 32767 is used: a one-ulp reciprocal keeps |qf - xa/yc| < 2^-7, so the floor
    // is exact or one off, which the correction below fixes (the IEEE division would cost ~12 instructions)
#if defined(__HIP_DEVICE_COMPILE__) && !AT2V_LEHMER_IEEE_DIV
    const float qf = (float)xa * __builtin_amdgcn_rcpf((float)yc);
#else
    const float qf = (float)xa / (float)yc;
#endif
    if (qf >= 32767.0f) break;                // keep q, cofactors and products inside 32 bits
    int32_t q = (int32_t)qf;
    int32_t r = xa - q * yc;  // fix the estimate to the exact floor (off by at most one)
    if (r < 0) {
      --q;
      r += yc;
    } else if (r >= yc) {
      ++q;
      r -= yc;
    }
    const int32_t r2 = xb - q * yd;  // Knuth's test: same quotient for the other end of the interval
    if (r2 < 0 || r2 >= yd) break;
    const int32_t nC = A - q * Cc, nD = B - q * D;
    if (nC >= 32768 || nC <= -32768 || nD >= 32768 || nD <= -32768) break;
    A = Cc;
    Cc = nC;
    B = D;
    D = nD;
    const int32_t ny = x - q * y;
    x = y;
    y = ny;
    ++steps;
  }
  A64 = A;
  B64 = B;
  C64 = Cc;
  D64 = D;
}

// dst = p a + q b for cofactors of opposite signs (or a zero one), known to be >= 0
AT2V_HD AT2V_INLINE void u256_lincomb(U256& dst, const U256& a, int64_t p, const U256& b, int64_t q) {
  U256 x, y;
#pragma unroll
  for (int i = 0; i < 8; ++i) x.w[i] = y.w[i] = 0;
  u256_addmul(x, a, (uint32_t)iabs64(p));
  u256_addmul(y, b, (uint32_t)iabs64(q));
  if (q <= 0) {  // p >= 0 >= q
    u256_sub(x, y);
    dst = x;
  } else {        // p <= 0 < q
    u256_sub(y, x);
    dst = y;
  }
}

// (ra, rb) <- (A ra + B rb, C ra + D rb); cofactor magnitudes add (signs alternate)
AT2V_HD AT2V_INLINE void lehmer_apply(U256& ra, U256& rb, U256& ma, U256& mb, int64_t A, int64_t B, int64_t Cc,
                                      int64_t D) {
  U256 na, nb;
  u256_lincomb(na, ra, A, rb, B);
  u256_lincomb(nb, ra, Cc, rb, D);
  U256 xa, xb;
#pragma unroll
  for (int i = 0; i < 8; ++i) xa.w[i] = xb.w[i] = 0;
  u256_addmul(xa, ma, (uint32_t)iabs64(A));
  u256_addmul(xa, mb, (uint32_t)iabs64(B));
  u256_addmul(xb, ma, (uint32_t)iabs64(Cc));
  u256_addmul(xb, mb, (uint32_t)iabs64(D));
  ra = na;
  rb = nb;
  ma = xa;
  mb = xb;
}

// One reduction round from (ra, rb, ma, mb) into a DIFFERENT set (na, nb, xa, xb): a Lehmer round, an exact step as
// the matrix (0 1; 1 -q), or (rare) the exact subtract-and-swap step. Writing into the other set lets the caller
// alternate two register sets (AT2V_LATTICE_PINGPONG) instead of copying the new state back every round.
AT2V_HD AT2V_INLINE void lattice_step(const U256& ra, const U256& rb, const U256& ma, const U256& mb, U256& na, U256& nb,
                                      U256& xa, U256& xb, int& idx, const U256& C) {
  int steps;
  int64_t mA, mB, mC, mD;
  lehmer_round32(steps, mA, mB, mC, mD, ra, rb, C);
  if (steps == 0) {  // exact step through the same apply when the double quotient is provably the floor
    const double ratio = u256_to_double(ra) / u256_to_double(rb);
    if (ratio < 2147483648.0) {
      const double fl = (double)(int64_t)ratio;
      const double fr = ratio - fl;
      if (fr > 1.0 / 65536 && fr < 1.0 - 1.0 / 65536) {
        mA = 0;
        mB = 1;
        mC = 1;
        mD = -(int64_t)fl;
        steps = 1;
      }
    }
  }
  if (steps > 0) {
    u256_lincomb(na, ra, mA, rb, mB);
    u256_lincomb(nb, ra, mC, rb, mD);
#pragma unroll
    for (int i = 0; i < 8; ++i) xa.w[i] = xb.w[i] = 0;
    u256_addmul(xa, ma, (uint32_t)iabs64(mA));
    u256_addmul(xa, mb, (uint32_t)iabs64(mB));
    u256_addmul(xb, ma, (uint32_t)iabs64(mC));
    u256_addmul(xb, mb, (uint32_t)iabs64(mD));
    idx += steps;
  } else {
    U256 r = ra, m = ma;
    euclid_reduce(r, m, rb, mb);  // r = ra mod rb, m = ma + q mb
    na = rb;
    xa = mb;
    nb = r;
    xb = m;
    ++idx;
  }
}

struct HalfScalars {
  uint32_t c0[8];   // c0 >= 0
  uint32_t c1[8];   // |c1| (odd)
  int c1_neg;       // sign of c1
  int bits;         // max(bitlen(c0), bitlen(|c1|))
};

// (c0, c1) for k < l: c0 = c1 * k (mod 8l), c1 odd, short. See the header comment.
AT2V_HD AT2V_INLINE void lattice_reduce(HalfScalars& out, const uint32_t k[8]) {
  const uint32_t n8[8] = AT2V_8L_WORDS;
  const uint32_t sq[8] = AT2V_SQRT8L_WORDS;
  U256 C;
  u256_set(C, sq);
  U256 ra, rb, ma, mb;
  u256_set(ra, n8);
  u256_set(rb, k);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    ma.w[i] = 0;
    mb.w[i] = i == 0;
  }
  int idx = 1;  // rb = r_idx; sign(t_idx) = (-1)^(idx+1)
#if AT2V_LATTICE_LEHMER == 2 && AT2V_LATTICE_PINGPONG
  {
    U256 sa, sb, sma, smb;
    int in_second = 0;
    for (int guard = 0; guard < 200 && u256_ge(rb, C); ++guard) {
      lattice_step(ra, rb, ma, mb, sa, sb, sma, smb, idx, C);
      if (!u256_ge(sb, C)) {
        in_second = 1;
        break;
      }
      lattice_step(sa, sb, sma, smb, ra, rb, ma, mb, idx, C);
    }
    if (in_second) {
      ra = sa;
      rb = sb;
      ma = sma;
      mb = smb;
    }
  }
#elif AT2V_LATTICE_LEHMER
  for (int guard = 0; guard < 400 && u256_ge(rb, C); ++guard) {
    int steps;
    int64_t mA, mB, mC, mD;
#if AT2V_LATTICE_LEHMER == 2
    lehmer_round32(steps, mA, mB, mC, mD, ra, rb, C);
#else
    lehmer_round(steps, mA, mB, mC, mD, ra, rb, C);
#endif
#if AT2V_LATTICE_EXACT_MATRIX
    if (steps == 0) {
      // One exact Euclid step as the cofactor matrix (0 1; 1 -q), so it runs through the same lehmer_apply as a
      // Lehmer round instead of a separate subtract-and-swap path (whose join copied the 4 x 8-word state). The
      // double quotient is taken only when it is provably the floor: q < 2^31 and the fraction at least 2^-16 away
      // from an integer (the two 256-bit -> double conversions and the division err by < 2^-48 relative, i.e.
      // < 2^-17 absolute here); otherwise (probability ~2^-15 per step) the exact path below runs.
      const double ratio = u256_to_double(ra) / u256_to_double(rb);
      if (ratio < 2147483648.0) {
        const double fl = (double)(int64_t)ratio;
        const double fr = ratio - fl;
        if (fr > 1.0 / 65536 && fr < 1.0 - 1.0 / 65536) {
          mA = 0;
          mB = 1;
          mC = 1;
          mD = -(int64_t)fl;
          steps = 1;
        }
      }
    }
#endif
    if (steps > 0) {
      lehmer_apply(ra, rb, ma, mb, mA, mB, mC, mD);
      idx += steps;
    } else {
      euclid_reduce(ra, ma, rb, mb);  // one exact multi-precision step (large quotient / near the threshold)
      const U256 tr = ra, tm = ma;
      ra = rb;
      ma = mb;
      rb = tr;
      mb = tm;
      ++idx;
    }
  }
#else
  for (int guard = 0; guard < 400 && u256_ge(rb, C); ++guard) {
    euclid_reduce(ra, ma, rb, mb);  // ra = r_{idx+1}, ma = m_{idx+1}
    const U256 tr = ra, tm = ma;
    ra = rb;
    ma = mb;
    rb = tr;
    mb = tm;
    ++idx;
  }
#endif
  // Candidates (all lattice vectors; keep the shortest with odd c1):
  //   (r_idx, t_idx), (r_{idx-1}, t_{idx-1}), and with one more Euclid step (r2, t2) = (r_{idx+1}, t_{idx+1}):
  //   (r2, t2), (r_idx + r2, t_idx + t2), (r_idx - r2, t_idx - t2). Signs alternate: sign(t_idx) =
  //   (-1)^(idx+1), t_{idx-1} and t2 have the opposite sign. rb = 0 only when k = 0 (then t_idx = 1).
  const int tb_neg = (idx & 1) == 0;
  U256 c0 = rb, c1 = mb;  // by value: per-lane selects, no pointers to registers
  int neg = tb_neg;
  int best = (mb.w[0] & 1u) ? imax(u256_bitlen(rb), u256_bitlen(mb)) : 1000;
  U256 r2 = ra, m2 = ma, sb = rb, db = rb, ms = ma, md = ma;
  int nonzero = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) nonzero |= rb.w[i] != 0;
  if (nonzero) {
    euclid_reduce(r2, m2, rb, mb);
    if (ma.w[0] & 1u) {
      const int b = imax(u256_bitlen(ra), u256_bitlen(ma));
      if (b < best) {
        c0 = ra;
        c1 = ma;
        neg = !tb_neg;
        best = b;
      }
    }
    if (m2.w[0] & 1u) {
      const int b = imax(u256_bitlen(r2), u256_bitlen(m2));
      if (b < best) {
        c0 = r2;
        c1 = m2;
        neg = !tb_neg;
        best = b;
      }
    }
    if ((mb.w[0] ^ m2.w[0]) & 1u) {
      u256_add(sb, r2);  // rb + r2 < 2 rb
      u256_sub(db, r2);  // rb - r2 > 0
      // |t_idx + t2| = |m2 - mb| (opposite signs), sign of the larger; |t_idx - t2| = mb + m2, sign of t_idx
      ms = m2;
      int s_neg = !tb_neg;
      if (u256_ge(ms, mb)) {
        u256_sub(ms, mb);
      } else {
        ms = mb;
        u256_sub(ms, m2);
        s_neg = tb_neg;
      }
      md = m2;
      const uint32_t carry = u256_add(md, mb);
      const int bs = imax(u256_bitlen(sb), u256_bitlen(ms));
      if (bs < best) {
        c0 = sb;
        c1 = ms;
        neg = s_neg;
        best = bs;
      }
      const int bd = carry ? 1000 : imax(u256_bitlen(db), u256_bitlen(md));
      if (bd < best) {
        c0 = db;
        c1 = md;
        neg = tb_neg;
        best = bd;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    out.c0[i] = c0.w[i];
    out.c1[i] = c1.w[i];
  }
  out.c1_neg = neg;
  // keep |c1| < 2^254 so its signed radix-16 recoding (64 digits) cannot carry out: |c1| < 8l always,
  // and for |c1| >= 2^254, c1 -> c1 - sign(c1) 8l keeps the congruence and the parity, |c1| <= 2^254 + 2^128
  U256 m;
#pragma unroll
  for (int i = 0; i < 8; ++i) m.w[i] = out.c1[i];
  if (m.w[7] >= 0x40000000u) {
    U256 n;
    u256_set(n, n8);
    u256_sub(n, m);
#pragma unroll
    for (int i = 0; i < 8; ++i) out.c1[i] = n.w[i];
    out.c1_neg = !out.c1_neg;
  }
  U256 a, b;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a.w[i] = out.c0[i];
    b.w[i] = out.c1[i];
  }
  out.bits = imax(u256_bitlen(a), u256_bitlen(b));
}

// t = c1 * s mod l (c1 signed, s < l)
AT2V_HD AT2V_INLINE void sc_mul_signed(uint32_t t[8], const HalfScalars& h, const uint32_t s[8]) {
  uint32_t x[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint64_t p = (uint64_t)h.c1[i] * s[j] + x[i + j] + carry;
      x[i + j] = (uint32_t)p;
      carry = p >> 32;
    }
    x[i + 8] = (uint32_t)carry;
  }
  sc_reduce512(t, x);  // |c1| < 2^255, s < 2^253: product < 2^508
  if (h.c1_neg) {      // t = l - t (t != 0)
    const uint32_t l[8] = AT2V_L_WORDS;
    uint32_t z = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) z |= t[i];
    uint64_t borrow = 0;
    uint32_t u[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint64_t d = (uint64_t)l[i] - t[i] - borrow;
      u[i] = (uint32_t)d;
      borrow = (d >> 63) & 1;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) t[i] = z ? u[i] : 0u;
  }
}

}  // namespace at2v
