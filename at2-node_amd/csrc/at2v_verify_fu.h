// at2v_verify_fu.h — per-lane half-size Ed25519 verify on the unsigned field (at2v_fu / at2v_gu).
//
// Same equation, checks and verdicts as verify_half (at2v_verify.h): accept <=> s < l, A decodes, R_bytes canonical and
// decodes, and V = [c1]R + [c0]A - [t]B = 0 with (c0, c1) from lattice_reduce(k) and t = c1 s mod l. Replaces, per
// record, drop::crypto::sign -> ed25519-dalek `PublicKey::verify` on every payload broadcast at
// /root/reference/src/bin/server/rpc.rs:275-284. What changes is the arithmetic: unsigned limbs with the carry chained
// through the MAD addend (tools/gen_fu.py), the A and R decodes as one interleaved pair of exponentiations, the two
// per-lane tables built as interleaved pairs.
//   TabP : store(e, gu_cached) / prefetch(e) / load_prefetched(gu_cached)   (per lane, e in 0..8)
//   TabB : prefetch(e) / load_prefetched(gu_niels)                          (shared, e in 0..2^15)
#pragma once
#include "at2v_comb.h"
#include "at2v_gu.h"
#include "at2v_verify.h"

namespace at2v {

// kCacheable: the per-sender A cache is on (at2v_opts.sender_cache). Then a_cached = 1 (wave-uniform: every lane of the
// wave found its A in the cache, confirmed byte for byte) means `ta` already holds the lane's [j]A table (the cache
// entry) and a_cached_ok is dalek's decode verdict for A; only R is decoded and only R's table is built. Everything the
// verdict depends on is still a function of (A, R||S, M) alone.
#ifndef AT2V_PARK_POINTS
#define AT2V_PARK_POINTS 0  // 1: decoded A and R parked in the table slots across SHA-512 / lattice (0: kept live)
#endif
// The A and R decodes and the two tables ran as interleaved pairs in round 2. One after the other they hold fewer live
// values: verify_kernel's spills fall from 146 to 75 VGPRs (scratch 688 -> 464 B/lane) and the kernel runs 2.2% faster
// (two A/B runs on two boxes, profiles/r03q, r03r). 1 = the round-2 interleaved forms (A/B).
#ifndef AT2V_DECODE_X2
#define AT2V_DECODE_X2 0
#endif
#ifndef AT2V_TABLES_X2
#define AT2V_TABLES_X2 0
#endif
// AT2V_TABLES_EARLY = 1: each point's table is built right after its decode, so no decoded point is live across SHA-512
// and the lattice reduction (80 words). R's table then holds [j](+R) and the sign of c1, known only after the reduction,
// is applied per digit in the ladder (one XOR into the entry's conditional negation). Spills 75 -> 56 VGPRs, yet 1.1%
// slower in an A/B (profiles/r03u): not the default. 0 = both tables after the reduction, from the decoded points kept
// live (or parked: AT2V_PARK_POINTS).
#ifndef AT2V_TABLES_EARLY
#define AT2V_TABLES_EARLY 0
#endif
// AT2V_DECODE_LATE = 1: A and R are decoded after SHA-512, the lattice reduction and the recoding, right before their
// tables, so only the 24 digit words (not the two decoded points, 80 words) are live across those phases. The verdict is
// the same conjunction of checks in another order; a lane whose decode fails may set the wave's window count, which only
// costs windows.
#ifndef AT2V_DECODE_LATE
#define AT2V_DECODE_LATE 0
#endif

// AT2V_DECODE_LOOP = 1 (round 5 experiment): the two decodes, and later the two table builds, as rolled loops over
// {A, R} (one code copy each; the decoded points parked in their table slots across SHA-512 and the lattice reduction,
// as AT2V_PARK_POINTS does). The comb kernel gained 6% from the same change to its per-record code.
#ifndef AT2V_DECODE_LOOP
#define AT2V_DECODE_LOOP 0
#endif

// AT2V_TAB_MADD = 1 (round 5): a table's base point is a decoded point, affine (Z = 1), so [j+1]P = [j]P + P is a mixed
// addition with P's affine Niels form (y+x, y-x, 2dxy; the two sums carried, as the B tables' entries are): 3 products
// instead of 4 per entry (D = Z1 * 2 Z2 becomes 2 Z1), 7 M fewer per table, 14 per verify. The operand classes are the
// ladder's own (gu_madd after gu_p1p1_to_p3 with a carried Niels point, tools/gen_fu.py check_group_law).
#ifndef AT2V_TAB_MADD
#define AT2V_TAB_MADD 1
#endif

// [j]P, j = 0..8, cached form, into tp (one table; the A/B form of the interleaved build). P1 is a decoded point (Z = 1).
template <class TabP>
AT2V_HD AT2V_INLINE void build_a_table_from(const gu_p3& P1, TabP& tp) {
  gu_cached c1, cj;
  gu_cached_identity(cj);
  tp.store(0, cj);
  gu_p3_to_cached(c1, P1);
  tp.store(1, c1);
  gu_p3 Q = P1;
#if AT2V_TAB_MADD
  gu_niels n1;
  n1.ypx = c1.YpX;
  fu_carry(n1.ypx);
  n1.ymx = c1.YmX;
  fu_carry(n1.ymx);
  n1.xy2d = c1.T2d;  // 2d T = 2d x y (Z = 1), a carried product
#endif
#pragma unroll 1
  for (int j = 2; j <= 8; ++j) {
    gu_p1p1 s;
#if AT2V_TAB_MADD
    gu_madd(s, Q, n1);
#else
    gu_add(s, Q, c1);
#endif
    gu_p1p1_to_p3(Q, s);
    gu_p3_to_cached(cj, Q);
    tp.store(j, cj);
  }
}

// kBW: width of the fixed-base windows. 16 (tb0 = [j]B, tb1 = [j 2^128]B, j <= 2^15, 4.2 MB each: the CPU backend, and
// the GPU kernels' default until round 6): 8 B windows, at ladder windows 0, 4, ..., 28, each adding two entries. 24
// (tb0 = [j]B, tb1 = [j 2^144]B, j <= 2^23, 1 GB each, shared per device: the throughput kernels since round 6,
// AT2V_LADDER_BW): t = sum e_k 2^(24 k), k = 0..10, 6 B windows at ladder windows 0, 6, ..., 30 adding e_k and e_(k+6):
// 12 mixed additions instead of 16 per verify (-28 M of 1195 M, 1.6% of the MACs), read at random from 2 GB.
template <bool kCacheable = false, int kBW = 16, class TabP, class TabB0, class TabB1, class MsgWord, class WaveMax,
          class Pace = NoPace>
AT2V_HD AT2V_INLINE int verify_half_fu(const uint32_t Rw[8], const uint32_t Aw[8], const uint32_t Sw[8], uint32_t len,
                                       MsgWord msgword, int policy, TabP& ta, TabP& tr, const TabB0& tb0,
                                       const TabB1& tb1, WaveMax wave_max, Pace&& pace = Pace(), int a_cached = 0,
                                       int a_cached_ok = 0) {
  // V1: s < l
  int ok = sc_is_canonical(Sw);
  if (policy == POLICY_LIBSODIUM_1_0_18) {
    ok &= !enc_small_order(Rw);
    ok &= enc_y_canonical(Aw) & !enc_small_order(Aw);
  }
  // V2: decode A and R; R must be canonical (y < p, not x = 0 with the sign bit)
#if !AT2V_DECODE_LATE && !AT2V_DECODE_LOOP
  gu_p3 A, R;
#endif
#if AT2V_DECODE_LOOP
  {
    int okd = 1;
#pragma unroll 1
    for (int q = (kCacheable && a_cached) ? 1 : 0; q < 2; ++q) {
      uint32_t W[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) W[i] = q ? Rw[i] : Aw[i];
      gu_p3 P;
      okd &= gu_frombytes(P, W);
      if (q) okd &= enc_y_canonical(Rw) & !(fu_iszero(P.X) & (int)(Rw[7] >> 31));
      TabP& tp = q ? tr : ta;
      tp.park(P);
    }
    ok &= okd;
    if (kCacheable && a_cached) ok &= a_cached_ok;
  }
#elif AT2V_DECODE_LATE
  // (after the reduction, below)
#elif AT2V_TABLES_EARLY
  // 1: both tables early; 2: A's table early, R kept live (its table after the reduction); 3: R's table early (sign of
  // c1 per digit), A kept live
  if (kCacheable && a_cached) {  // [j]A comes from the cache entry
    ok &= a_cached_ok;
  } else {
    ok &= gu_frombytes(A, Aw);
    if (AT2V_TABLES_EARLY != 3) build_a_table_from(A, ta);
  }
  ok &= gu_frombytes(R, Rw);
  ok &= enc_y_canonical(Rw);
  ok &= !(fu_iszero(R.X) & (int)(Rw[7] >> 31));
  if (AT2V_TABLES_EARLY != 2) build_a_table_from(R, tr);
#else
  if (kCacheable && a_cached) {
    ok &= gu_frombytes(R, Rw) & a_cached_ok;
  } else {
#if AT2V_DECODE_X2
    int okd[2];
    gu_frombytes_x2(A, Aw, R, Rw, okd);
    ok &= okd[0] & okd[1];
#else
    ok &= gu_frombytes(A, Aw);
    ok &= gu_frombytes(R, Rw);
#endif
  }
  ok &= enc_y_canonical(Rw);
  ok &= !(fu_iszero(R.X) & (int)(Rw[7] >> 31));
#endif
#if AT2V_PARK_POINTS && !AT2V_TABLES_EARLY && !AT2V_DECODE_LATE && !AT2V_DECODE_LOOP
  // A and R are not used again until the tables are built (after SHA-512, the lattice reduction and the recoding), and
  // holding their 80 words through those phases is what makes the compiler spill (one scratch reload and wait per
  // word, ~50 of them at the table build). Park them in the lanes' table slots (entry 8, written last by the build)
  // with 20 fire-and-forget stores; reload them with 20 loads and one wait where the build starts.
  if (!(kCacheable && a_cached)) ta.park(A);
  tr.park(R);
#endif
  AT2V_PHASE(1);
  pace.mark(10);
  // V3: k = SHA-512(R || A || M) mod l
  uint32_t k[8];
  {
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
  }
  AT2V_PHASE(5);
  pace.mark(3);
  HalfScalars hs;
  lattice_reduce(hs, k);
  AT2V_PHASE(7);
  pace.mark(3);
  uint32_t t[8];
  sc_mul_signed(t, hs, Sw);
  static_assert(kBW == 16 || kBW == 24, "fixed-base window");
  constexpr int kTdWords = kBW == 16 ? 8 : 12;  // 24: 11 digits + a zero digit (stored 2^23) for the 12th entry
  uint32_t c0d[8], c1d[8], td[kTdWords];
  sc_recode4_hi8(c0d, hs.c0);
  sc_recode4_hi8(c1d, hs.c1);
  if constexpr (kBW == 16) {
    sc_recode16(td, t);
  } else {
    sc_recode_w<24>(td, t);
    td[11] = 1u << 23;
  }
  // 64 signed radix-16 digits hold values < 2^255 (the reduction keeps max(|c0|, |c1|) < 2^253); a lane
  // that would need a 65th window fails closed
  ok &= hs.bits <= 255;
  const int nw_lane = ok ? hs.bits / 4 + 1 : 0;
  int nw = wave_max(nw_lane);
  // B digits sit at windows 0, 4, ..., 28 (kBW 16) or 0, 6, ..., 30 (24): the top window (no B digit) lies above them
  constexpr int kNwMin = kBW == 16 ? 30 : 32;
  nw = nw < kNwMin ? kNwMin : nw;
  AT2V_PHASE(2);
  pace.mark(1);

  // tables [j]A and [j](+-R), j = 0..8: one after the other (AT2V_TABLES_X2 = 0, the default since round 3: the pair's
  // extra live registers cost more in spills than its ILP gains, profiles/r03q), or as one interleaved pair
#if AT2V_DECODE_LOOP
  const int rflip = 0;
#pragma unroll 1
  for (int q = (kCacheable && a_cached) ? 1 : 0; q < 2; ++q) {
    TabP& tp = q ? tr : ta;
    gu_p3 P;
    tp.unpark(P);
    if (q && hs.c1_neg) {
      fu_neg(P.X, P.X, FU_KC);
      fu_carry(P.X);
      fu_neg(P.T, P.T, FU_KC);
      fu_carry(P.T);
    }
    build_a_table_from(P, tp);
  }
#elif AT2V_DECODE_LATE
  const int rflip = 0;
  if (kCacheable && a_cached) {  // [j]A comes from the cache entry
    ok &= a_cached_ok;
  } else {
    gu_p3 A;
    ok &= gu_frombytes(A, Aw);
    build_a_table_from(A, ta);
  }
  {
    gu_p3 R;
    ok &= gu_frombytes(R, Rw);
    ok &= enc_y_canonical(Rw);
    ok &= !(fu_iszero(R.X) & (int)(Rw[7] >> 31));
    if (hs.c1_neg) {
      fu_neg(R.X, R.X, FU_KC);
      fu_carry(R.X);
      fu_neg(R.T, R.T, FU_KC);
      fu_carry(R.T);
    }
    build_a_table_from(R, tr);
  }
#elif AT2V_TABLES_EARLY
  const int rflip = AT2V_TABLES_EARLY != 2 ? hs.c1_neg : 0;  // [c1]R = [|c1|](-R) when c1 < 0: flips every R digit
  if (AT2V_TABLES_EARLY == 2) {
    if (hs.c1_neg) {
      fu_neg(R.X, R.X, FU_KC);
      fu_carry(R.X);
      fu_neg(R.T, R.T, FU_KC);
      fu_carry(R.T);
    }
    build_a_table_from(R, tr);
  }
  if (AT2V_TABLES_EARLY == 3 && !(kCacheable && a_cached)) build_a_table_from(A, ta);
#else
  const int rflip = 0;
#if AT2V_PARK_POINTS
  if (!(kCacheable && a_cached)) ta.unpark(A);
  tr.unpark(R);
#endif
  if (hs.c1_neg) {
    fu_neg(R.X, R.X, FU_KC);
    fu_carry(R.X);
    fu_neg(R.T, R.T, FU_KC);
    fu_carry(R.T);
  }
  if (kCacheable && a_cached) {  // [j]A comes from the cache entry: build [j](+-R) alone
    build_a_table_from(R, tr);
  } else {
#if AT2V_TABLES_X2
    gu_cached ca1, cr1, cj;
    gu_cached_identity(cj);
    ta.store(0, cj);
    tr.store(0, cj);
    gu_p3_to_cached(ca1, A);
    gu_p3_to_cached(cr1, R);
    ta.store(1, ca1);
    tr.store(1, cr1);
    gu_p3 PA = A, PR = R;
#pragma unroll 1
    for (int j = 2; j <= 8; ++j) {
      gu_p1p1 sa, sr;
      gu_add(sa, PA, ca1);
      gu_add(sr, PR, cr1);
      gu_p1p1_to_p3(PA, sa);
      gu_p1p1_to_p3(PR, sr);
      gu_p3_to_cached(cj, PA);
      ta.store(j, cj);
      gu_p3_to_cached(cj, PR);
      tr.store(j, cj);
    }
#else
    build_a_table_from(A, ta);
    build_a_table_from(R, tr);
#endif
  }
#endif  // AT2V_TABLES_EARLY
  AT2V_PHASE(3);
  pace.mark(4);

  // shared doubling chain over windows nw-1 .. 0:
  //   acc = 16 acc + a_i A + r_i (+-R) + [4 | i, i < 32] (-t_{i/4} [2^(16 i/4)]B - t_{8+i/4} [2^(128+16 i/4)]B)
  gu_p2 R2;
  gu_p3 R3;
  gu_p1p1 tt;
  gu_cached ca;
  gu_niels nb;
  auto digit4 = [](const uint32_t d[8], int i) -> int { return (int)((sel8(d, i >> 3) >> (4 * (i & 7))) & 15) - 7; };
  {
    const int i = nw - 1;
    const int da = digit4(c0d, i), dr = digit4(c1d, i);
    ta.prefetch(da < 0 ? -da : da);
    tr.prefetch(dr < 0 ? -dr : dr);
    gu_p3_identity(R3);
    ta.load_prefetched(ca);
    gu_cached_cneg(ca, da < 0);
    gu_add(tt, R3, ca);
    gu_p1p1_to_p3(R3, tt);
    tr.load_prefetched(ca);
    gu_cached_cneg(ca, (dr < 0) ^ rflip);
    gu_add(tt, R3, ca);
    gu_p1p1_to_p2(R2, tt);
  }
  // The digit words live in a private array that LLVM keeps in scratch: a uniform-index read is a scratch load with an
  // SGPR offset. Read at the start of the window that needs them, their round trip (together with the pacing load
  // issued just before) stalled every window on s_waitcnt vmcnt(0) (SQ_WAIT_ANY 12.8% of wave cycles, profiles/r02q).
  // AT2V_DIGIT_AHEAD=1: the words of the NEXT window's A/R digits and this window's B digits are loaded at the window
  // start, before the LDS-DMA prefetches (vmcnt counts in issue order, so waiting for them never waits for the
  // prefetches), and first used a window (A/R) or four doublings (B) later. 0 = the old placement (A/B).
#ifndef AT2V_DIGIT_AHEAD
#define AT2V_DIGIT_AHEAD 1
#endif
#if AT2V_DIGIT_AHEAD
  uint32_t wa = sel8(c0d, (nw - 2) >> 3), wr = sel8(c1d, (nw - 2) >> 3);
#endif
  for (int i = nw - 2; i >= 0; --i) {
    const int bk = kBW == 16 ? i >> 2 : i / 6;  // the B digit index of a B window
    const bool bwin = kBW == 16 ? (i & 3) == 0 && i < 32 : bk * 6 == i && i < 36;
    int e0 = 0, e1 = 0;
#if AT2V_DIGIT_AHEAD
    // before the pacing store/load of this window: the wait for wa/wr must not wait for them
    int da, dr;
    AT2V_PROBE(pace.probe[0], {
      da = (int)((wa >> (4 * (i & 7))) & 15) - 7;
      dr = (int)((wr >> (4 * (i & 7))) & 15) - 7;
#if defined(__HIP_DEVICE_COMPILE__)
      asm volatile("" ::"v"(da), "v"(dr) : "memory");  // da, dr exist before the pacing store below is issued
#endif
    });
    pace.window();
    wa = sel8(c0d, (i - 1) >> 3);  // i = 0: index -1 selects word 0, unused
    wr = sel8(c1d, (i - 1) >> 3);
    // used only when bwin: kBW 16, the words holding digits i/4 and 8 + i/4; 24, digits i/6 and 6 + i/6 themselves
    const uint32_t wt0 = kBW == 16 ? sel8(td, i >> 3) : seln<kTdWords>(td, bk);
    const uint32_t wt1 = kBW == 16 ? sel8(td, 4 + (i >> 3)) : seln<kTdWords>(td, 6 + bk);
#else
    pace.window();
    const int da = digit4(c0d, i), dr = digit4(c1d, i);
#endif
    ta.prefetch(da < 0 ? -da : da);  // both land while the window's four doublings run
    tr.prefetch(dr < 0 ? -dr : dr);
    for (int r = 0; r < 3; ++r) {
      gu_p2_dbl(tt, R2);
      gu_p1p1_to_p2(R2, tt);
    }
    gu_p2_dbl(tt, R2);
    gu_p1p1_to_p3(R3, tt);
    AT2V_PROBE(pace.probe[1], pace.mid());
    if (bwin) {  // -t digits: j = i/4 (table [j]B) and 8 + i/4 (table [j 2^128]B); kBW 24: i/6 and 6 + i/6
#if AT2V_DIGIT_AHEAD
      if constexpr (kBW == 16) {
        e0 = (1 << 15) - (int)((wt0 >> (16 * ((i >> 2) & 1))) & 0xffff);
        e1 = (1 << 15) - (int)((wt1 >> (16 * ((i >> 2) & 1))) & 0xffff);
      } else {
        e0 = (1 << 23) - (int)wt0;
        e1 = (1 << 23) - (int)wt1;
      }
#else
      static_assert(kBW == 16, "the 24-bit fixed-base windows read their digits ahead");
      e0 = (1 << 15) - (int)((sel8(td, i >> 3) >> (16 * ((i >> 2) & 1))) & 0xffff);
      e1 = (1 << 15) - (int)((sel8(td, 4 + (i >> 3)) >> (16 * ((i >> 2) & 1))) & 0xffff);
#endif
    }
    ta.load_prefetched(ca);
    if (bwin) tb0.prefetch(e0 < 0 ? -e0 : e0);  // into A's stage, now consumed
    gu_cached_cneg(ca, da < 0);
    gu_add(tt, R3, ca);
    gu_p1p1_to_p3(R3, tt);
    tr.load_prefetched(ca);
    if (bwin) tb1.prefetch(e1 < 0 ? -e1 : e1);  // into R's stage
    gu_cached_cneg(ca, (dr < 0) ^ rflip);
    gu_add(tt, R3, ca);
    if (bwin) {
      gu_p1p1_to_p3(R3, tt);
      tb0.load_prefetched(nb);
      gu_niels_cneg(nb, e0 < 0);
      gu_madd(tt, R3, nb);
      gu_p1p1_to_p3(R3, tt);
      tb1.load_prefetched(nb);
      gu_niels_cneg(nb, e1 < 0);
      gu_madd(tt, R3, nb);
    }
    gu_p1p1_to_p2(R2, tt);
  }
  AT2V_PHASE(4);
  // V == identity: X = 0 and Y = Z
  fu d;
  fu_sub(d, R2.Y, R2.Z, FU_KC);
  return ok & fu_iszero(R2.X) & fu_iszero(d);
}

// ---------------------------------------------------------------------------------------------------------------
// Two lanes per signature (the low-latency kernel). Side 0 owns A, side 1 owns R: each lane decodes
// one point, builds one table, and runs its half of the shared-window chain,
//   side 0: P0 = [c0]A - [t_lo]B          side 1: P1 = [c1]R - [t_hi 2^128]B   (t = t_lo + 2^128 t_hi),
// so a lane does four doublings and one addition per window instead of two additions, and one of the two
// fixed-base additions. V = P0 + P1 is then formed from the partner's cached point (verify_pair_combine). The
// SHA-512 and the lattice reduction run on both lanes (same code, no divergence). Returns this side's checks:
// side 0 V1, the policy pre-checks and A's decode; side 1 R's decode and canonicity. The signature is valid iff both
// sides' checks pass and V is the identity.
//   TabP : this lane's table of its point;  TabB : this lane's fixed-base table ([j]B on side 0, [j 2^128]B on side 1)
template <class TabP, class TabB, class MsgWord, class WaveMax>
AT2V_HD AT2V_INLINE int verify_pair_part(int side, const uint32_t Rw[8], const uint32_t Aw[8], const uint32_t Sw[8],
                                         uint32_t len, MsgWord msgword, int policy, TabP& tp, const TabB& tb,
                                         WaveMax wave_max, gu_p3& out) {
  int ok;
  gu_p3 P;
  if (side == 0) {
    ok = sc_is_canonical(Sw);
    if (policy == POLICY_LIBSODIUM_1_0_18) {
      ok &= !enc_small_order(Rw);
      ok &= enc_y_canonical(Aw) & !enc_small_order(Aw);
    }
  } else {
    ok = enc_y_canonical(Rw);
  }
  ok &= gu_frombytes(P, side ? Rw : Aw);
  if (side) ok &= !(fu_iszero(P.X) & (int)(Rw[7] >> 31));
  AT2V_PHASE(1);
  uint32_t k[8];
  {
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
  }
  AT2V_PHASE(5);
  HalfScalars hs;
  lattice_reduce(hs, k);
  AT2V_PHASE(7);
  uint32_t t[8];
  sc_mul_signed(t, hs, Sw);
  uint32_t cd[8], td[8];
  sc_recode4_hi8(cd, side ? hs.c1 : hs.c0);
  sc_recode16(td, t);
  ok &= hs.bits <= 255;
  // the window count must cover both sides' scalars: every lane computes the same hs, so its own bits suffice
  const int nw_lane = hs.bits <= 255 ? hs.bits / 4 + 1 : 0;
  int nw = wave_max(nw_lane);
  nw = nw < 30 ? 30 : nw;  // the top window (no B digit) must lie above the B windows 0, 4, ..., 28
  AT2V_PHASE(2);
  if (side && hs.c1_neg) {
    fu_neg(P.X, P.X, FU_KC);
    fu_carry(P.X);
    fu_neg(P.T, P.T, FU_KC);
    fu_carry(P.T);
  }
  build_a_table_from(P, tp);
  AT2V_PHASE(3);
  gu_p2 R2;
  gu_p3 R3;
  gu_p1p1 tt;
  gu_cached ca;
  gu_niels nb;
  auto digit4 = [](const uint32_t d[8], int i) -> int { return (int)((sel8(d, i >> 3) >> (4 * (i & 7))) & 15) - 7; };
  {
    const int d = digit4(cd, nw - 1);
    tp.prefetch(d < 0 ? -d : d);
    gu_p3_identity(R3);
    tp.load_prefetched(ca);
    gu_cached_cneg(ca, d < 0);
    gu_add(tt, R3, ca);
    gu_p1p1_to_p2(R2, tt);
  }
  for (int i = nw - 2; i >= 0; --i) {
    const int d = digit4(cd, i);
    tp.prefetch(d < 0 ? -d : d);  // lands while the window's four doublings run
    for (int r = 0; r < 3; ++r) {
      gu_p2_dbl(tt, R2);
      gu_p1p1_to_p2(R2, tt);
    }
    gu_p2_dbl(tt, R2);
    gu_p1p1_to_p3(R3, tt);
    const bool bwin = (i & 3) == 0 && i < 32;
    int e = 0;
    if (bwin)  // -t digit j = i/4 of this side's half: table [j]B (side 0) or [j 2^128]B (side 1)
      e = (1 << 15) - (int)((sel8(td, (side ? 4 : 0) + (i >> 3)) >> (16 * ((i >> 2) & 1))) & 0xffff);
    tp.load_prefetched(ca);
    if (bwin) tb.prefetch(e < 0 ? -e : e);
    gu_cached_cneg(ca, d < 0);
    gu_add(tt, R3, ca);
    if (bwin) {
      gu_p1p1_to_p3(R3, tt);
      tb.load_prefetched(nb);
      gu_niels_cneg(nb, e < 0);
      gu_madd(tt, R3, nb);
    }
    if (i > 0) gu_p1p1_to_p2(R2, tt);
  }
  gu_p1p1_to_p3(out, tt);
  AT2V_PHASE(4);
  return ok;
}

// V = mine + partner (the partner's point in cached form) == identity: in p1p1 (E, H, G, F), x = E/G and y = H/F,
// so V = (0, 1) <=> E = 0 and H = F
AT2V_HD AT2V_INLINE int verify_pair_combine(const gu_p3& mine, const gu_cached& partner) {
  gu_p1p1 v;
  gu_add(v, mine, partner);
  fu d;
  fu_sub(d, v.T, v.Y, FU_K2C);  // F + K - H: H = B + A is a sum of two carried elements, F may exceed FU_KC
  return fu_iszero(v.X) & fu_iszero(d);
}

}  // namespace at2v

namespace at2v {

// [c]P from the table [j]P (tp, j = 0..8) over windows nw-1..0 of c's signed radix-16 digits (sc_recode4_hi8 nibbles,
// d_i + 7): four doublings and one addition per window; flip = 1 negates every digit (the scalar's sign, applied per
// entry because the table was built before the sign was known).
template <class TabP>
AT2V_HD AT2V_INLINE void split_side_ladder(gu_p3& out, const uint32_t cd[8], int nw, int flip, TabP& tp) {
  gu_p2 R2;
  gu_p3 R3;
  gu_p1p1 tt;
  gu_cached ca;
  auto digit4 = [](const uint32_t d[8], int i) -> int { return (int)((sel8(d, i >> 3) >> (4 * (i & 7))) & 15) - 7; };
  {
    const int d = digit4(cd, nw - 1);
    tp.prefetch(d < 0 ? -d : d);
    gu_p3_identity(R3);
    tp.load_prefetched(ca);
    gu_cached_cneg(ca, (d < 0) ^ flip);
    gu_add(tt, R3, ca);
    gu_p1p1_to_p2(R2, tt);
  }
  for (int i = nw - 2; i >= 0; --i) {
    const int d = digit4(cd, i);
    tp.prefetch(d < 0 ? -d : d);  // lands while the window's four doublings run
    for (int r = 0; r < 3; ++r) {
      gu_p2_dbl(tt, R2);
      gu_p1p1_to_p2(R2, tt);
    }
    gu_p2_dbl(tt, R2);
    gu_p1p1_to_p3(R3, tt);
    tp.load_prefetched(ca);
    gu_cached_cneg(ca, (d < 0) ^ flip);
    gu_add(tt, R3, ca);
    if (i > 0) gu_p1p1_to_p2(R2, tt);
  }
  gu_p1p1_to_p3(out, tt);
}

// ---------------------------------------------------------------------------------------------------------------
// The half-size check split over four waves (the low-latency comb kernel's path for chunks whose senders are not all
// cached): V = [c0]A + [c1]R - [t]B = 0 as in verify_half_fu (§4b), with the parts that do not depend on
// each other run side by side —
//   wave 0: split_a_side (V1, policy pre-checks, decode A, [j]A)   then split_side_ladder over c0 with [j]A
//   wave 1: split_r_side (R canonical, decode R, [j]R)              then split_side_ladder over |c1| with [j]R, sign of c1
//   wave 2: split_scalars (SHA-512 -> k, lattice, t)               then split_neg_tb: -[t]B from the comb of B
// and split_combine on wave 0. The verdict is exactly verify_half_fu's: the same checks, the same group element V (any
// evaluation of the three products gives it), the same identity test.

template <class TabP>
AT2V_HD AT2V_INLINE int split_a_side(gu_p3& A, const uint32_t Rw[8], const uint32_t Aw[8], const uint32_t Sw[8],
                                     int policy, TabP& tp) {
  int ok = sc_is_canonical(Sw);
  if (policy == POLICY_LIBSODIUM_1_0_18) {
    ok &= !enc_small_order(Rw);
    ok &= enc_y_canonical(Aw) & !enc_small_order(Aw);
  }
  ok &= gu_frombytes(A, Aw);
  build_a_table_from(A, tp);
  return ok;
}

template <class TabP>
AT2V_HD AT2V_INLINE int split_r_side(const uint32_t Rw[8], TabP& tp) {
  gu_p3 R;
  int ok = enc_y_canonical(Rw);
  ok &= gu_frombytes(R, Rw);
  ok &= !(fu_iszero(R.X) & (int)(Rw[7] >> 31));
  build_a_table_from(R, tp);
  return ok;
}

// digits of c0 and |c1| (sc_recode4_hi8), t = c1 s mod l (sc_recode16), the sign of c1 and the lane's window count;
// returns 0 for a lane whose scalars would need a 65th window (fails closed, as verify_half_fu)
template <class MsgWord>
AT2V_HD AT2V_INLINE int split_scalars(uint32_t c0d[8], uint32_t c1d[8], uint32_t td[kBCombLatDigitWords], int& c1_neg,
                                      int& nw_lane,
                                      const uint32_t Rw[8], const uint32_t Aw[8], const uint32_t Sw[8], uint32_t len,
                                      MsgWord msgword) {
  uint32_t k[8];
  {
    uint32_t pre[16];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      pre[q] = Rw[q];
      pre[8 + q] = Aw[q];
    }
    uint64_t h[8];
    sha512_msg<16>(h, pre, len, msgword);
    uint32_t hw[16];
    sha512_digest_words(hw, h);
    sc_reduce512(k, hw);
  }
  HalfScalars hs;
  lattice_reduce(hs, k);
  uint32_t t[8];
  sc_mul_signed(t, hs, Sw);
  sc_recode4_hi8(c0d, hs.c0);
  sc_recode4_hi8(c1d, hs.c1);
  bcomb_recode<kBCombLatBits>(td, t);  // (the low-latency comb of B's digits: -[t]B comes from it, split_neg_tb)
  c1_neg = hs.c1_neg;
  const int ok = hs.bits <= 255;
  nw_lane = ok ? hs.bits / 4 + 1 : 0;
  return ok;
}

// -[t]B in cached form, from the comb of B (TabBC: prefetch(stage, i, j) / load_prefetched(stage, gu_niels&))
template <class TabBC>
AT2V_HD AT2V_INLINE void split_neg_tb(gu_cached& out, const uint32_t* td, const TabBC& tb) {
  gu_p3 P;
  gu_p3_identity(P);
  comb_sum<false>(P, td, 0, BCombGeom<TabBC::kBits>::kPos, tb);
  gu_p3_to_cached(out, P);
  gu_cached_cneg(out, 1);
}

// V = P0 + P1 + (-[t]B) == identity (P1 and -[t]B in cached form)
AT2V_HD AT2V_INLINE int split_combine(const gu_p3& P0, const gu_cached& P1, const gu_cached& nTB) {
  gu_p1p1 t;
  gu_add(t, P0, P1);
  gu_p3 S;
  gu_p1p1_to_p3(S, t);
  return verify_pair_combine(S, nTB);
}

// Per-sender cache entry (at2v_opts.sender_cache; AT2 senders repeat, accounts/account.rs:36-43): dalek's decode verdict
// for A and the table [j]A, j = 0..8, built by exactly the steps verify_half_fu uses for its own [j]A, in the layout it
// reads through `ta`. Returns the decode verdict (the table is unused when it is 0).
template <class TabP>
AT2V_HD AT2V_INLINE int build_a_table(const uint32_t Aw[8], TabP& ta) {
  gu_p3 A;
  const int ok = gu_frombytes(A, Aw);
  build_a_table_from(A, ta);
  return ok;
}

}  // namespace at2v
