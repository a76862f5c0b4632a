// at2v_comb.h — verify from per-key comb tables (at2v_opts.sender_comb).
//
// AT2 senders issue consecutive sequences (/root/reference/src/bin/server/accounts/account.rs:36-43): one public key A
// signs many payloads. For such a key the device keeps a comb of -A, C[i][j] = [j 2^(10i)](-A) for i = 0..25, j = 0..512
// (affine Niels, or cached form with AT2V_COMB_NIELS=0), next to the context's comb of B, D[i][j] = [j 2^(Wi)]B for
// i = 0..kBCombPos-1, j = 0..2^(W-1) (affine Niels; W = 24: 11 positions).
// Then dalek's point R' = [k](-A) + [s]B is a sum of 26 + 11 table entries, no doublings:
//   k = sum_i e_i 2^(10i), e_i in [-512, 511] (sc_recode_w) ->  [k](-A) = sum_i +-C[i][|e_i|]
//   s = sum_i f_i 2^(Wi), f_i in [-2^(W-1), 2^(W-1)) (bcomb_recode) ->  [s]B = sum_i +-D[i][|f_i|]
// and the verdict is dalek's own comparison, enc(R') == R_bytes (the full-length form, DESIGN.md §4: no lattice
// reduction, no decode of R). Any correct evaluation of [k](-A) + [s]B is the same group element, so the verdicts are
// those of the ladder kernels (and of the oracle), for every key the comb was built from, small-order and mixed-order
// keys included; a key that fails dalek's decode has verdict 0 whatever the comb holds.
//
// Cost per verify: 37 mixed additions (7 M; 42 with W = 16) + one inversion (254 S + 11 M; shared by four records in the throughput
// kernel) + SHA-512, against the half-size ladder's 2 exponentiations + 2 tables + 33 windows: ~5x fewer
// multiplications. The comb of one key is 26 x 513 x 128 B = 1.7 MB (10-bit windows), built once (comb_build_lane).
//   TabC  : prefetch(stage, i, j) / load_prefetched(stage, CombEntry&)   entry C[i][j] of this lane's key
//   TabBC : prefetch(stage, i, j) / load_prefetched(stage, gu_niels&)    entry D[i][j]
// Two stages alternate: the entry of the next addition is fetched while this one is computed. The low-latency kernel
// splits one record's work over four waves (decode R | 11 B entries | SHA-512 + 13 A entries | SHA-512 + 13 A entries)
// and compares R' with the decoded R projectively (comb_check_split).
#pragma once
#include "at2v_gu.h"
#include "at2v_verify.h"

namespace at2v {

// A comb window: signed radix-2^w digits of k (w = AT2V_COMB_BITS). w = 10 (default): 26 positions x 513 entries, 1.7 MB
// per key; w = 8: 32 positions x 129 entries, 660 KB per key, 6 additions more per verify (368.4 vs 399.9 M/s on 64-sender
// traffic, profiles/r03z).
#ifndef AT2V_COMB_BITS
#define AT2V_COMB_BITS 10
#endif
constexpr int kCombBits = AT2V_COMB_BITS;
static_assert(kCombBits >= 4 && kCombBits <= 15, "A comb window");
constexpr int kCombPos = (254 + kCombBits - 1) / kCombBits;    // positions (sc_recode_w's digit count)
constexpr int kCombEntries = (1 << (kCombBits - 1)) + 1;        // j = 0..2^(w-1) per position (j = 0: the identity)
// Comb builders: a launch with few new keys gives each key a 256-thread block, 8 lanes per position (kCombWideLog2: the
// latency of a first-seen sender); one with many gives each key a wave, 2 lanes per position (kCombNarrowLog2: fewer
// redundant position chains when the waves outnumber the SIMDs). Both build the same points (representations differ).
constexpr int kCombWideLog2 = 3, kCombNarrowLog2 = 1;
static_assert(kCombBits - 1 - kCombWideLog2 >= 1, "comb builder parts");
static_assert((kCombPos << kCombWideLog2) <= 256, "one 256-thread block builds a key's comb");
static_assert((kCombPos << kCombNarrowLog2) <= 64, "one wave builds a key's comb");
// new keys per launch up to which the wide builder runs (a 256-thread block per key). A build block holds its CU for
// the ~1 ms of a comb's 250-doubling position chain, and no verify block fits beside it (they take the whole register
// file), so AT2V_COMB_WIDE_MAX bounds the CUs builds take from the verify kernels: above it, one wave per key (four keys
// per block).
#ifndef AT2V_COMB_WIDE_MAX
#define AT2V_COMB_WIDE_MAX 8  // 256 (a block per key up to 256 keys): Zipf / 4x-capacity legs 2-3% slower (profiles/r05zf)
#endif
constexpr int kCombWideMaxKeys = AT2V_COMB_WIDE_MAX;
constexpr int kCombDigitWords = (kCombPos + 1) / 2;             // k's digits, two 16-bit fields per word
// The combs of B: signed radix-2^W digits of s. Every context with combs holds two: W = 16 (16 positions x (2^15 + 1)
// entries, 67 MB, MALL-resident), read by the low-latency kernel and every other comb path, and W = 20 (13 positions,
// 872 MB) for the hit-list kernel, three additions fewer per record. AT2V_CTX_BCOMB_WIDE makes the latter W = 24 (11
// positions x (2^23 + 1) entries, 11.8 GB of the 288 GB HBM, five fewer). 64-sender traffic: 514.0 / 535.4 / 551.8 M/s
// with W = 16 / 20 / 24 in the hit-list kernel (profiles/r05v/abcomb_bcomb_bits.txt). W = 24 is opt-in for its memory
// and its 0.75 s build; config 5's latency is the same with it in every node process (profiles/r05zn).
#ifndef AT2V_BCOMB_BITS
#define AT2V_BCOMB_BITS 24
#endif
template <int W>
struct BCombGeom {
  static_assert(W == 16 || W == 20 || W == 24, "B comb window");
  static constexpr int kPos = (254 + W - 1) / W;                // positions
  static constexpr int kEntries = (1 << (W - 1)) + 1;           // j = 0..2^(W-1)
  static constexpr int kDigitWords = W == 16 ? 8 : kPos;        // 16: two halfword digits per word
  static constexpr size_t kBytes = (size_t)kPos * kEntries * 128;
};
constexpr int kBCombBits = AT2V_BCOMB_BITS;  // the wide comb of B (AT2V_CTX_BCOMB_WIDE)
constexpr int kBCombMidBits = 20;            // every comb context's throughput comb of B (872 MB)
constexpr int kBCombLatBits = 16;            // every comb context's low-latency comb of B (67 MB)
constexpr int kBCombPos = BCombGeom<kBCombBits>::kPos;
constexpr int kBCombEntries = BCombGeom<kBCombBits>::kEntries;
constexpr int kBCombDigitWords = BCombGeom<kBCombBits>::kDigitWords;
constexpr int kBCombLatPos = BCombGeom<kBCombLatBits>::kPos;
constexpr int kBCombLatDigitWords = BCombGeom<kBCombLatBits>::kDigitWords;
// A-comb entry form. 1 (default since round 4): affine Niels (y+x, y-x, 2dxy), 30 words in 8 granules = one 128-byte
// line, mixed additions (7 M); the builder normalises its lane's entries with one inversion (Montgomery's trick).
// 0: cached (Y+X, Y-X, 2Z, 2dT), 40 words in 10 granules (two or three lines), 8 M additions.
#ifndef AT2V_COMB_NIELS
#define AT2V_COMB_NIELS 1
#endif
constexpr bool kCombNiels = AT2V_COMB_NIELS != 0;
template <bool kNiels> struct CombEntrySel { using type = gu_cached; };
template <> struct CombEntrySel<true> { using type = gu_niels; };
using CombEntry = CombEntrySel<kCombNiels>::type;
constexpr int kCombGranules = kCombNiels ? 8 : 10;
constexpr int kCombWords = kCombGranules * 4;
constexpr size_t kCombBytes = (size_t)kCombPos * kCombEntries * kCombGranules * 16;  // per key

// R' (p2) encoded as dalek's CompressedEdwardsY (y canonical, sign bit = low bit of canonical x) == R_bytes
AT2V_HD AT2V_INLINE int gu_encode_eq(const gu_p2& P, const uint32_t Rw[8]) {
  fu zi, x, y;
  fu_invert(zi, P.Z);
  fu_mulc(x, P.X, zi);
  fu_mulc(y, P.Y, zi);
  uint32_t enc[8], xb[8];
  fu_tobytes(enc, y);
  fu_tobytes(xb, x);
  enc[7] ^= (xb[0] & 1u) << 31;
  int eq = 1;
#pragma unroll
  for (int i = 0; i < 8; ++i) eq &= enc[i] == Rw[i];
  return eq;
}

// enc(P) == R_bytes with 1/Z given (P in p2 or p3: x = X/Z, y = Y/Z)
template <class P>
AT2V_HD AT2V_INLINE int gu_encode_eq_zi(const P& p, const fu& zi, const uint32_t Rw[8]) {
  fu x, y;
  fu_mulc(x, p.X, zi);
  fu_mulc(y, p.Y, zi);
  uint32_t enc[8], xb[8];
  fu_tobytes(enc, y);
  fu_tobytes(xb, x);
  enc[7] ^= (xb[0] & 1u) << 31;
  int eq = 1;
#pragma unroll
  for (int i = 0; i < 8; ++i) eq &= enc[i] == Rw[i];
  return eq;
}

// Checks that need no point arithmetic: V1 (s < l), A's decode verdict (held with the comb), libsodium's pre-rejects.
AT2V_HD AT2V_INLINE int comb_prechecks(const uint32_t Rw[8], const uint32_t Aw[8], const uint32_t Sw[8], int policy,
                                       int a_ok) {
  int ok = sc_is_canonical(Sw) & a_ok;
  if (policy == POLICY_LIBSODIUM_1_0_18) {
    ok &= !enc_small_order(Rw);
    ok &= enc_y_canonical(Aw) & !enc_small_order(Aw);
  }
  return ok;
}

// V3 and the recoding of k: kd = signed radix-2^w digits of SHA-512(R || A || M) mod l, e_i + 2^(w-1) in 16-bit fields
template <class MsgWord>
AT2V_HD AT2V_INLINE void comb_k_digits(uint32_t kd[kCombDigitWords], const uint32_t Rw[8], const uint32_t Aw[8],
                                       uint32_t len, MsgWord msgword) {
  uint32_t k[8];
  uint32_t pre[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    pre[i] = Rw[i];
    pre[8 + i] = Aw[i];
  }
  uint64_t h[8];
  sha512_msg<16>(h, pre, len, msgword);
  uint32_t hw[16];
  sha512_digest_words(hw, h);
  sc_reduce512(k, hw);
  uint32_t d[kCombPos];
  sc_recode_w<kCombBits>(d, k);
#pragma unroll
  for (int q = 0; q < kCombDigitWords; ++q)
    kd[q] = d[2 * q] | (2 * q + 1 < kCombPos ? d[2 * q + 1] << 16 : 0u);
}

AT2V_HD AT2V_INLINE int comb_adigit(const uint32_t kd[kCombDigitWords], int i) {
  return (int)((seln<kCombDigitWords>(kd, i >> 1) >> (16 * (i & 1))) & 0xffff) - (1 << (kCombBits - 1));
}
template <int W = kBCombBits>
AT2V_HD AT2V_INLINE int comb_bdigit(const uint32_t* sd, int i) {
  if constexpr (W == 16) return (int)((sel8(sd, i >> 1) >> (16 * (i & 1))) & 0xffff) - 0x8000;
  else return (int)seln<BCombGeom<W>::kDigitWords>(sd, i) - (1 << (W - 1));
}
// s (or t) -> the digits of a W-bit comb of B
template <int W = kBCombBits>
AT2V_HD AT2V_INLINE void bcomb_recode(uint32_t out[BCombGeom<W>::kDigitWords], const uint32_t s[8]) {
  if constexpr (W == 16) sc_recode16(out, s);
  else sc_recode_w<W>(out, s);
}

// acc += sum over positions i in [i0, i1) of the signed entry C[i][e_i] (A comb, kAComb: CombEntry) or D[i][f_i] (B
// comb of Tab::kBits-bit windows, affine Niels). The entry of addition m + 1 is fetched (into the other stage) while m
// is computed.
template <bool kAComb, class Tab>
AT2V_HD AT2V_INLINE void comb_sum(gu_p3& acc, const uint32_t* dig, int i0, int i1, const Tab& tab) {
  auto digit = [&](int i) {
    if constexpr (kAComb) return comb_adigit(dig, i);
    else return comb_bdigit<Tab::kBits>(dig, i);
  };
  gu_p1p1 t;
  int e = digit(i0);
  tab.prefetch(0, i0, e < 0 ? -e : e);
#pragma unroll 1
  for (int i = i0; i < i1; i += 2) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {  // stage h holds entry i + h
      const int m = i + h;
      if (m >= i1) break;  // an odd count (wave-uniform)
      const int en = m + 1 < i1 ? digit(m + 1) : 0;
      if constexpr (kAComb && !kCombNiels) {
        gu_cached ca;
        tab.load_prefetched(h, ca);
        if (m + 1 < i1) tab.prefetch(h ^ 1, m + 1, en < 0 ? -en : en);
        gu_cached_cneg(ca, e < 0);
        gu_add(t, acc, ca);
      } else {
        gu_niels nb;
        tab.load_prefetched(h, nb);
        if (m + 1 < i1) tab.prefetch(h ^ 1, m + 1, en < 0 ? -en : en);
        gu_niels_cneg(nb, e < 0);
        gu_madd(t, acc, nb);
      }
      gu_p1p1_to_p3(acc, t);
      e = en;
    }
  }
}

// R' = [k](-A) + [s]B of one record from the combs (V3 + V4 of the full-length form): the point, not yet encoded
template <class TabC, class TabBC, class MsgWord>
AT2V_HD AT2V_INLINE void comb_point(gu_p3& acc, const uint32_t Rw[8], const uint32_t Aw[8], const uint32_t Sw[8],
                                    uint32_t len, MsgWord msgword, const TabC& tc, const TabBC& tb) {
  uint32_t kd[kCombDigitWords], sd[BCombGeom<TabBC::kBits>::kDigitWords];
  comb_k_digits(kd, Rw, Aw, len, msgword);
  bcomb_recode<TabBC::kBits>(sd, Sw);
  gu_p3_identity(acc);
  comb_sum<true>(acc, kd, 0, kCombPos, tc);
  comb_sum<false>(acc, sd, 0, BCombGeom<TabBC::kBits>::kPos, tb);
}

// dalek-1.x verify of one record from the comb of its key (one lane per record: the throughput path).
template <class TabC, class TabBC, class MsgWord>
AT2V_HD AT2V_INLINE int verify_comb_fu(const uint32_t Rw[8], const uint32_t Aw[8], const uint32_t Sw[8], uint32_t len,
                                       MsgWord msgword, int policy, int a_ok, const TabC& tc, const TabBC& tb) {
  const int ok = comb_prechecks(Rw, Aw, Sw, policy, a_ok);
  uint32_t kd[kCombDigitWords], sd[BCombGeom<TabBC::kBits>::kDigitWords];
  comb_k_digits(kd, Rw, Aw, len, msgword);
  bcomb_recode<TabBC::kBits>(sd, Sw);
  AT2V_PHASE(2);
  // V4: R' = [k](-A) + [s]B as the sum of the kCombPos A entries and the kBCombPos B entries
  gu_p3 acc;
  gu_p3_identity(acc);
  comb_sum<true>(acc, kd, 0, kCombPos, tc);
  comb_sum<false>(acc, sd, 0, BCombGeom<TabBC::kBits>::kPos, tb);
  AT2V_PHASE(4);
  // V5/V6: dalek compares the compressed R' with the 32 bytes of R
  gu_p2 Rp;
  gu_p3_to_p2(Rp, acc);
  return ok & gu_encode_eq(Rp, Rw);
}

// The low-latency split (verify_comb_lat_kernel: one wave per part, on different SIMDs): R decoded on its own instead
// of R' encoded (no inversion after the sums), R' = Pa0 + Pa1 + Pb from the partial sums, compared projectively.
// enc(R') == R_bytes <=> R_bytes is canonical (y < p, not x = 0 with the sign bit set), decodes, and dec(R_bytes) = R'
// (DESIGN.md §4b step 5), so the verdict is dalek's.
AT2V_HD AT2V_INLINE int comb_decode_r(gu_p3& R, const uint32_t Rw[8]) {
  int ok = gu_frombytes(R, Rw);
  ok &= enc_y_canonical(Rw);
  ok &= !(fu_iszero(R.X) & (int)(Rw[7] >> 31));
  return ok;
}
AT2V_HD AT2V_INLINE int comb_check_split(const gu_p3& R, const gu_p3& Pa0, const gu_p3& Pa1, const gu_p3& Pb) {
  gu_cached c;
  gu_p1p1 t;
  gu_p3 S;
  gu_p3_to_cached(c, Pa1);
  gu_add(t, Pa0, c);
  gu_p1p1_to_p3(S, t);
  gu_p3_to_cached(c, Pb);
  gu_add(t, S, c);
  gu_p2 P;
  gu_p1p1_to_p2(P, t);
  // R = (x, y, 1, xy): X = x Z and Y = y Z
  fu u, d;
  fu_mulc(u, R.X, P.Z);
  fu_sub(d, P.X, u, FU_KC);
  const int ex = fu_iszero(d);
  fu_mulc(u, R.Y, P.Z);
  fu_sub(d, P.Y, u, FU_KC);
  return ex & fu_iszero(d);
}

// One lane's share of the comb of key A, with 2^kPartsLog2 lanes per position: position pos (0..kCombPos-1), part h ->
// entries j = kPart h + 1 .. kPart (h + 1) (kPart = 2^(w-1-kPartsLog2)) of C[pos][j] = [j 2^(w pos)](-A), written through
// mem.put(j, words) (kCombWords words in CombEntry's layout); the h = 0 lane also writes j = 0 (the identity). kCombPos
// 2^kPartsLog2 lanes (pos = lane >> kPartsLog2, h = the low bits) build the whole comb; a lane with pos >= kCombPos
// writes nothing. Every lane decodes A (dalek rules) and returns the decode verdict; an undecodable A yields a comb that
// no verdict depends on. Per lane: (kCombPos - 1) w doublings (the position chain), log2(kPart) doublings and h
// additions to the part's first multiple, kPart additions (w = 10: 8 parts, 256 doublings and at most 71 additions; 2
// parts, 258 doublings and at most 257 additions). Affine entries (kCombNiels) take two passes over the lane's own
// entries: pass 1 writes (X pi', Y pi', Z) with pi' the product of the earlier Z's, one inversion of the product of all
// of them, pass 2 (backwards, mem.get) turns each into (y+x, y-x, 2dxy) with x = X pi' / pi: 8 M more per entry.
template <class Mem>
AT2V_HD AT2V_INLINE void comb_put_fu3(Mem& mem, int j, const fu& a, const fu& b, const fu& c) {
  uint32_t w[kCombWords];
#pragma unroll
  for (int q = 0; q < 10; ++q) {
    w[q] = a.v[q];
    w[10 + q] = b.v[q];
    w[20 + q] = c.v[q];
  }
#pragma unroll
  for (int q = 30; q < kCombWords; ++q) w[q] = 0;
  mem.put(j, w);
}

template <int kPartsLog2, class Mem>
AT2V_HD AT2V_INLINE int comb_build_lane(const uint32_t Aw[8], int pos, int h, Mem& mem) {
  constexpr int kPartBits = kCombBits - 1 - kPartsLog2;
  constexpr int kPart = 1 << kPartBits;
  gu_p3 P;
  const int ok = gu_frombytes(P, Aw);
  fu_neg(P.X, P.X, FU_KC);  // -A
  fu_carry(P.X);
  fu_neg(P.T, P.T, FU_KC);
  fu_carry(P.T);
  if (pos >= kCombPos) return ok;
  // Pi = [2^(w pos)](-A): every lane runs the (kCombPos - 1) x w doublings and keeps its position's point
  gu_p3 Pi = P, Q = P;
  gu_p2 Q2;
  gu_p1p1 t;
#pragma unroll 1
  for (int r = 1; r < kCombPos; ++r) {
    gu_p3_to_p2(Q2, Q);
#pragma unroll 1
    for (int d = 0; d < kCombBits - 1; ++d) {
      gu_p2_dbl(t, Q2);
      gu_p1p1_to_p2(Q2, t);
    }
    gu_p2_dbl(t, Q2);
    gu_p1p1_to_p3(Q, t);
    if (r == pos) Pi = Q;
  }
  gu_cached c1;
  gu_p3_to_cached(c1, Pi);
  // first multiple of this part: [kPart h + 1]Pi = Pi + h [kPart]Pi
  gu_p3 S = Pi;
  {
    gu_p2 D2;
    gu_p3_to_p2(D2, Pi);
#pragma unroll 1
    for (int d = 0; d < kPartBits - 1; ++d) {
      gu_p2_dbl(t, D2);
      gu_p1p1_to_p2(D2, t);
    }
    gu_p2_dbl(t, D2);
    gu_p3 D;
    gu_p1p1_to_p3(D, t);
    gu_cached dc;
    gu_p3_to_cached(dc, D);
#pragma unroll 1
    for (int m = 0; m < h; ++m) {
      gu_add(t, S, dc);
      gu_p1p1_to_p3(S, t);
    }
  }
  const int j0 = kPart * h + 1;
  if constexpr (!kCombNiels) {
    if (h == 0) {
      gu_cached id;
      gu_cached_identity(id);
      mem.put(0, reinterpret_cast<const uint32_t*>(&id));
    }
    gu_cached cj;
#pragma unroll 1
    for (int m = 0; m < kPart; ++m) {
      gu_p3_to_cached(cj, S);
      mem.put(j0 + m, reinterpret_cast<const uint32_t*>(&cj));
      if (m + 1 < kPart) {
        gu_add(t, S, c1);
        gu_p1p1_to_p3(S, t);
      }
    }
  } else {
    if (h == 0) {
      fu one, zero;
      fu_1(one);
      fu_0(zero);
      comb_put_fu3(mem, 0, one, one, zero);  // identity: y+x = 1, y-x = 1, 2dxy = 0
    }
    fu pi;  // pass 1: pi = Z_0 ... Z_m; entry m holds (X_m pi_(m-1), Y_m pi_(m-1), Z_m)
#pragma unroll 1
    for (int m = 0; m < kPart; ++m) {
      if (m == 0) {
        comb_put_fu3(mem, j0, S.X, S.Y, S.Z);
        pi = S.Z;
      } else {
        fu xp, yp;
        fu_mulc(xp, S.X, pi);
        fu_mulc(yp, S.Y, pi);
        comb_put_fu3(mem, j0 + m, xp, yp, S.Z);
        fu_mulc(pi, pi, S.Z);
      }
      if (m + 1 < kPart) {
        gu_add(t, S, c1);
        gu_p1p1_to_p3(S, t);
      }
    }
    fu inv;  // 1 / pi_m, m from the last entry down
    fu_invert(inv, pi);
#pragma unroll 1
    for (int m = kPart - 1; m >= 0; --m) {
      uint32_t w[kCombWords];
      mem.get(j0 + m, w);
      fu xp, yp, z, x, y;
#pragma unroll
      for (int q = 0; q < 10; ++q) {
        xp.v[q] = w[q];
        yp.v[q] = w[10 + q];
        z.v[q] = w[20 + q];
      }
      fu_mulc(x, xp, inv);
      fu_mulc(y, yp, inv);
      fu_mulc(inv, inv, z);
      gu_niels n;
      fu_add(n.ypx, y, x);
      fu_carry(n.ypx);
      fu_sub(n.ymx, y, x, FU_KC);
      fu_carry(n.ymx);
      fu xy;
      fu_mulc(xy, x, y);
      fu_mulc(n.xy2d, xy, FU_D2);
      comb_put_fu3(mem, j0 + m, n.ypx, n.ymx, n.xy2d);
    }
  }
  return ok;
}

}  // namespace at2v
