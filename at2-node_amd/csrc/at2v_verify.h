// at2v_verify.h — per-lane Ed25519 verify, dalek-1.x semantics (SURVEY.md Appendix A V1–V6).
//
// Replaces, per record, the call drop::crypto::sign → ed25519-dalek `PublicKey::verify` that
// sieve/murmur make on every payload broadcast at /root/reference/src/bin/server/rpc.rs:275-284
// (consumed already-verified at rpc.rs:156-173).
//
// Double-scalar multiplication R' = [k](-A) + [s]B uses one shared doubling chain with
// wavefront-uniform fixed windows (every lane adds at the same positions, no divergence):
//   k : 64 signed radix-16 digits  in [-8, 8]     -> table [0..8](-A), cached form, per lane (global scratch)
//   s : ceil(254/WB) signed radix-2^WB digits (WB = 16, 20 or 24) -> table [0..2^(WB-1)]B, affine Niels,
//       in global memory (L2/MALL), entries prefetched into LDS by LDS-DMA
//   R = sum_i 16^i (k_i(-A) + [WB/4 | i] s_{4i/WB} B), Horner from i = 63: 252 doublings, 64 + ceil(254/WB)
//   additions.
// Any correct evaluation of [k](-A) + [s]B yields the same group element, so verdicts are
// identical to dalek's NAF-5/NAF-8 vartime ladder (the oracle restates that one).
#pragma once
#include "at2v_ge.h"
#include "at2v_lattice.h"
#include "at2v_sc.h"
#include "at2v_sha512.h"

// Phase-timing hook (tools/phase_bench.hip defines it to accumulate s_memtime deltas per wave; the
// product build compiles it away).
#ifndef AT2V_PHASE
#define AT2V_PHASE(k)
#endif
// s_waitcnt probe (tools/phase_bench built with -DAT2V_WAIT_PROBE): `acc += s_memtime cycles spent in stmt`; acc is a
// member of a kernel-scope object (a table or the pacer), so it stays in registers. Product builds: just stmt.
#if defined(AT2V_WAIT_PROBE) && defined(__HIP_DEVICE_COMPILE__)
#define AT2V_PROBE(acc, stmt)                                   \
  do {                                                          \
    const unsigned long long t0_ = __builtin_amdgcn_s_memtime(); \
    stmt;                                                       \
    (acc) += __builtin_amdgcn_s_memtime() - t0_;                \
  } while (0)
#else
#define AT2V_PROBE(acc, stmt) stmt
#endif

namespace at2v {

enum { POLICY_DALEK_V1 = 0, POLICY_LIBSODIUM_1_0_18 = 1 };

// uniform-index select from an N-word register array (avoids scratch for a runtime index)
template <int N>
AT2V_HD AT2V_INLINE uint32_t seln(const uint32_t* w, int j) {
  uint32_t r = w[0];
#pragma unroll
  for (int m = 1; m < N; ++m) r = (j == m) ? w[m] : r;
  return r;
}
AT2V_HD AT2V_INLINE uint32_t sel8(const uint32_t w[8], int j) { return seln<8>(w, j); }

// y-encoding (sign bit ignored) is canonical, i.e. y < p (libsodium ge25519_is_canonical)
AT2V_HD AT2V_INLINE int enc_y_canonical(const uint32_t s[8]) {
  const uint32_t top = s[7] & 0x7fffffffu;
  const int hi_all = (top == 0x7fffffffu) & (s[6] == 0xffffffffu) & (s[5] == 0xffffffffu) & (s[4] == 0xffffffffu) &
                     (s[3] == 0xffffffffu) & (s[2] == 0xffffffffu) & (s[1] == 0xffffffffu);
  return !(hi_all & (s[0] >= 0xffffffedu));
}

// y-encoding (sign bit masked) is in libsodium 1.0.18's small-order blocklist
AT2V_HD AT2V_INLINE int enc_small_order(const uint32_t s[8]) {
  int hit = 0;
#pragma unroll
  for (int b = 0; b < 7; ++b) {
    int eq = 1;
#pragma unroll
    for (int i = 0; i < 8; ++i) eq &= ((i == 7 ? (s[i] & 0x7fffffffu) : s[i]) == AT2V_SMALL_ORDER_Y[b][i]);
    hit |= eq;
  }
  return hit;
}

// [s]B for a reduced scalar s < l: Horner over 32 signed radix-256 digits, 8 doublings per digit
template <class TabB>
AT2V_HD AT2V_INLINE void ge_scalarmult_base(ge_p2& out, const uint32_t s[8], const TabB& tb) {
  uint32_t sd[8];
  sc_recode8(sd, s);
  ge_p3 R3;
  ge_p1p1 t;
  ge_niels nb;
  ge_p3_identity(R3);
  ge_p2 R2;
  for (int j = 31; j >= 0; --j) {
    if (j != 31) {
      for (int r = 0; r < 7; ++r) {
        ge_p2_dbl(t, R2);
        ge_p1p1_to_p2(R2, t);
      }
      ge_p2_dbl(t, R2);
      ge_p1p1_to_p3(R3, t);
    }
    const int e = (int)((sd[j >> 2] >> (8 * (j & 3))) & 255) - 128;
    tb.load(e < 0 ? -e : e, nb);
    ge_niels_cneg(nb, e < 0);
    ge_madd(t, R3, nb);
    ge_p1p1_to_p2(R2, t);
  }
  out = R2;
}

// Table access policies.
//   TabA: void store(int e, const ge_cached&); void load(int e, ge_cached&);  (per lane, e in 0..8)
//         void prefetch(int e); void load_prefetched(ge_cached&)   (asynchronous load of one entry)
//   TabB: void prefetch(int e); void load_prefetched(ge_niels&)               (shared, e in 0..2^(WB-1))
// WB = bits per fixed-base window (16, 20 or 24): s gets ceil(254/WB) signed digits, one every WB/4
// radix-16 windows, against a table [0..2^(WB-1)]B.
// V1..V4: checks, decode, hash, ladder. Returns the checks' verdict; R' = [k](-A) + [s]B in Rp.
template <int WB, class TabA, class TabB, class MsgWord>
AT2V_HD AT2V_INLINE int verify_ladder(ge_p2& Rp, const uint32_t Rw[8], const uint32_t Aw[8], const uint32_t Sw[8],
                                      uint32_t len, MsgWord msgword, int policy, TabA& ta, const TabB& tb) {
  // V1: s < l
  int ok = sc_is_canonical(Sw);
  if (policy == POLICY_LIBSODIUM_1_0_18) {
    ok &= !enc_small_order(Rw);
    ok &= enc_y_canonical(Aw) & !enc_small_order(Aw);
  }
  // V2: decode A (dalek rules)
  ge_p3 A;
  ok &= ge_frombytes(A, Aw);
  AT2V_PHASE(1);
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
    sha512_prefixed<16>(h, pre, len, msgword);
    uint32_t hw[16];
    sha512_digest_words(hw, h);
    sc_reduce512(k, hw);
  }
  constexpr int ND = ScWin<WB>::ND, WW = WB / 4;  // s digits; radix-16 windows per s digit
  static_assert(WB % 4 == 0 && (ND - 1) * WW <= 62, "s digits must sit on radix-16 windows below the top");
  uint32_t kd[8], sd[ND];
  sc_recode4(kd, k);
  sc_recode_w<WB>(sd, Sw);
  AT2V_PHASE(2);

  // table [j](-A), j = 0..8
  fe_neg(A.X, A.X);
  fe_neg(A.T, A.T);
  {
    ge_cached c1, cj;
    ge_cached_identity(cj);
    ta.store(0, cj);
    ge_p3_to_cached(c1, A);
    ta.store(1, c1);
    ge_p3 P = A;
    for (int j = 2; j <= 8; ++j) {
      ge_p1p1 t;
      ge_add(t, P, c1);
      ge_p1p1_to_p3(P, t);
      ge_p3_to_cached(cj, P);
      ta.store(j, cj);
    }
  }

  AT2V_PHASE(3);
  // V4: shared doubling chain over 64 radix-16 windows
  ge_p2 R2;
  ge_p3 R3;
  ge_p1p1 t;
  ge_cached ca;
  ge_niels nb;
  {  // top window i = 63 (odd: no B digit)
    const int d = (int)(kd[7] >> 28) - 8;
    ge_p3_identity(R3);
    ta.load(d < 0 ? -d : d, ca);
    ge_cached_cneg(ca, d < 0);
    ge_add(t, R3, ca);
    ge_p1p1_to_p2(R2, t);
  }
  for (int i = 62; i >= 0; --i) {
    const int d = (int)((sel8(kd, i >> 3) >> (4 * (i & 7))) & 15) - 8;
    ta.prefetch(d < 0 ? -d : d);  // both tables land while the window's four doublings run
    int e = 0;
    const bool bwin = (i % WW) == 0 && i / WW < ND;  // s digit j = i / WW (radix 2^WB)
    if (bwin) {
      e = (int)seln<ND>(sd, i / WW) - (1 << (WB - 1));
      tb.prefetch(e < 0 ? -e : e);
    }
    for (int r = 0; r < 3; ++r) {
      ge_p2_dbl(t, R2);
      ge_p1p1_to_p2(R2, t);
    }
    ge_p2_dbl(t, R2);
    ta.load_prefetched(ca);
    ge_p1p1_to_p3(R3, t);
    ge_cached_cneg(ca, d < 0);
    ge_add(t, R3, ca);
    if (bwin) {
      ge_p1p1_to_p3(R3, t);
      tb.load_prefetched(nb);
      ge_niels_cneg(nb, e < 0);
      ge_madd(t, R3, nb);
    }
    ge_p1p1_to_p2(R2, t);
  }
  Rp = R2;
  AT2V_PHASE(4);
  return ok;
}

// V5/V6: enc(R') with 1/Z given, compared with the 32 bytes of R (re-read by the caller, not kept live
// across the ladder)
AT2V_HD AT2V_INLINE int verify_finish(const ge_p2& Rp, const fe& zinv, const uint32_t Rr[8]) {
  fe x, y;
  fe_mul(x, Rp.X, zinv);
  fe_mul(y, Rp.Y, zinv);
  uint32_t enc[8], xb[8];
  fe_tobytes(enc, y);
  fe_tobytes(xb, x);
  enc[7] ^= (xb[0] & 1u) << 31;
  int eq = 1;
#pragma unroll
  for (int i = 0; i < 8; ++i) eq &= enc[i] == Rr[i];
  return eq;
}

template <int WB, class TabA, class TabB, class MsgWord, class RLoad>
AT2V_HD AT2V_INLINE int verify_core(const uint32_t Rw[8], const uint32_t Aw[8], const uint32_t Sw[8], uint32_t len,
                                    MsgWord msgword, int policy, TabA& ta, const TabB& tb, RLoad rload) {
  ge_p2 Rp;
  const int ok = verify_ladder<WB>(Rp, Rw, Aw, Sw, len, msgword, policy, ta, tb);
  fe zinv;
  fe_invert(zinv, Rp.Z);
  uint32_t Rr[8];
  rload(Rr);
  return ok & verify_finish(Rp, zinv, Rr);
}

// ---------------------------------------------------------------------------------------------------
// Half-size verification (tools/halfscalar_proto.py). Same verdicts as verify_core:
//   accept  <=>  s < l, A decodes, R_bytes canonical and decodes, and V = [c1]R + [c0]A - [t]B = 0,
// with (c0, c1) from lattice_reduce(k) (c0 = c1 k mod 8l, c1 odd) and t = c1 s mod l. V = [c1](R - R')
// for R' = [s]B - [k]A exactly (every point has [8l]P = 0), and [c1] is injective on E (c1 odd, 0 < |c1|
// < l), so V = 0 <=> R = R' <=> (R_bytes canonical) enc(R') == R_bytes. The doubling chain covers only
// max(|c0|, |c1|) ~ 2^128 (wave maximum, >= 29 windows): ~128 doublings instead of 252, two variable-base
// tables (A, +-R) and two fixed-base tables [j]B, [j 2^128]B (16-bit windows, t split at bit 128).
//   TabP : store(e, cached) / prefetch(e) / load_prefetched(cached)   (per lane, e in 0..8)
//   TabB : prefetch(e) / load_prefetched(niels)                       (shared, e in 0..2^15)
//   WaveMax : int(int) -> maximum over the lanes that verify together (identity on the host)
//   Pace : mark(units) after each phase, window() at each ladder window start, mid() after its doublings
//          (progress, ~1 unit per window; NoPace = none)
struct NoPace {
  AT2V_HD AT2V_INLINE void mark(uint32_t) {}
  AT2V_HD AT2V_INLINE void window() {}
  AT2V_HD AT2V_INLINE void mid() {}
};
template <class TabP, class TabB0, class TabB1, class MsgWord, class WaveMax, class Pace = NoPace>
AT2V_HD AT2V_INLINE int verify_half(const uint32_t Rw[8], const uint32_t Aw[8], const uint32_t Sw[8], uint32_t len,
                                    MsgWord msgword, int policy, TabP& ta, TabP& tr, const TabB0& tb0,
                                    const TabB1& tb1, WaveMax wave_max, Pace&& pace = Pace()) {
  // V1: s < l
  int ok = sc_is_canonical(Sw);
  if (policy == POLICY_LIBSODIUM_1_0_18) {
    ok &= !enc_small_order(Rw);
    ok &= enc_y_canonical(Aw) & !enc_small_order(Aw);
  }
  // V2: decode A; R must be canonical (y < p, not x = 0 with the sign bit) and decode
  ge_p3 A, R;
  ok &= ge_frombytes(A, Aw);
  ok &= enc_y_canonical(Rw);
  ok &= ge_frombytes(R, Rw);
  ok &= !(fe_iszero(R.X) & (int)(Rw[7] >> 31));
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
    sha512_prefixed<16>(h, pre, len, msgword);
    uint32_t hw[16];
    sha512_digest_words(hw, h);
    sc_reduce512(k, hw);
  }
  AT2V_PHASE(5);
  pace.mark(3);
  // half-size scalars
  HalfScalars hs;
  lattice_reduce(hs, k);
  AT2V_PHASE(7);
  pace.mark(3);
  uint32_t t[8];
  sc_mul_signed(t, hs, Sw);
  uint32_t c0d[8], c1d[8], td[8];
  sc_recode4_hi8(c0d, hs.c0);
  sc_recode4_hi8(c1d, hs.c1);
  sc_recode16(td, t);
  // 64 signed radix-16 digits hold values < 2^255. The reduction returns max(|c0|, |c1|) <= max(k, ~2^128) < 2^253
  // (tests/test_lattice_host.py), so this guard never fires; if it did, the lane fails closed
  // instead of running a 65th window on a truncated digit string.
  ok &= hs.bits <= 255;
  const int nw_lane = ok ? hs.bits / 4 + 1 : 0;  // windows for values < 2^(4 nw - 1); <= 64
  int nw = wave_max(nw_lane);
  nw = nw < 30 ? 30 : nw;  // B digits sit at windows 0, 4, ..., 28: the top window (no B digit) must lie above them
  AT2V_PHASE(2);
  pace.mark(1);

  // tables [j]A and [j](+-R), j = 0..8
  if (hs.c1_neg) {
    fe_neg(R.X, R.X);
    fe_neg(R.T, R.T);
  }
#pragma unroll 1
  for (int side = 0; side < 2; ++side) {
    const ge_p3& P0 = side ? R : A;
    TabP& tp = side ? tr : ta;
    ge_cached c1, cj;
    ge_cached_identity(cj);
    tp.store(0, cj);
    ge_p3_to_cached(c1, P0);
    tp.store(1, c1);
    ge_p3 P = P0;
    for (int j = 2; j <= 8; ++j) {
      ge_p1p1 tt;
      ge_add(tt, P, c1);
      ge_p1p1_to_p3(P, tt);
      ge_p3_to_cached(cj, P);
      tp.store(j, cj);
    }
  }
  AT2V_PHASE(3);
  pace.mark(4);

  // shared doubling chain over windows nw-1 .. 0:
  //   acc = 16 acc + a_i A + r_i (+-R) + [4 | i, i < 32] (-t_{i/4} [2^(16 i/4)]B - t_{8+i/4} [2^(128+16 i/4)]B)
  ge_p2 R2;
  ge_p3 R3;
  ge_p1p1 tt;
  ge_cached ca;
  ge_niels nb;
  auto digit4 = [](const uint32_t d[8], int i) -> int { return (int)((sel8(d, i >> 3) >> (4 * (i & 7))) & 15) - 7; };
  {
    const int i = nw - 1;
    const int da = digit4(c0d, i), dr = digit4(c1d, i);
    ta.prefetch(da < 0 ? -da : da);
    tr.prefetch(dr < 0 ? -dr : dr);
    ge_p3_identity(R3);
    ta.load_prefetched(ca);
    ge_cached_cneg(ca, da < 0);
    ge_add(tt, R3, ca);
    ge_p1p1_to_p3(R3, tt);
    tr.load_prefetched(ca);
    ge_cached_cneg(ca, dr < 0);
    ge_add(tt, R3, ca);
    ge_p1p1_to_p2(R2, tt);
  }
  for (int i = nw - 2; i >= 0; --i) {
    pace.window();
    const int da = digit4(c0d, i), dr = digit4(c1d, i);
    ta.prefetch(da < 0 ? -da : da);  // both land while the window's four doublings run
    tr.prefetch(dr < 0 ? -dr : dr);
    for (int r = 0; r < 3; ++r) {
      ge_p2_dbl(tt, R2);
      ge_p1p1_to_p2(R2, tt);
    }
    ge_p2_dbl(tt, R2);
    ge_p1p1_to_p3(R3, tt);
    pace.mid();
    const bool bwin = (i & 3) == 0 && i < 32;
    int e0 = 0, e1 = 0;
    if (bwin) {  // -t digits j = i/4 (table [j]B) and 8 + i/4 (table [j 2^128]B)
      e0 = (1 << 15) - (int)((sel8(td, i >> 3) >> (16 * ((i >> 2) & 1))) & 0xffff);
      e1 = (1 << 15) - (int)((sel8(td, 4 + (i >> 3)) >> (16 * ((i >> 2) & 1))) & 0xffff);
    }
    ta.load_prefetched(ca);
    if (bwin) tb0.prefetch(e0 < 0 ? -e0 : e0);  // into A's stage, now consumed
    ge_cached_cneg(ca, da < 0);
    ge_add(tt, R3, ca);
    ge_p1p1_to_p3(R3, tt);
    tr.load_prefetched(ca);
    if (bwin) tb1.prefetch(e1 < 0 ? -e1 : e1);  // into R's stage
    ge_cached_cneg(ca, dr < 0);
    ge_add(tt, R3, ca);
    if (bwin) {
      ge_p1p1_to_p3(R3, tt);
      tb0.load_prefetched(nb);
      ge_niels_cneg(nb, e0 < 0);
      ge_madd(tt, R3, nb);
      ge_p1p1_to_p3(R3, tt);
      tb1.load_prefetched(nb);
      ge_niels_cneg(nb, e1 < 0);
      ge_madd(tt, R3, nb);
    }
    ge_p1p1_to_p2(R2, tt);
  }
  AT2V_PHASE(4);
  // V == identity: X = 0 and Y = Z
  fe d;
  fe_sub(d, R2.Y, R2.Z);
  return ok & fe_iszero(R2.X) & fe_iszero(d);
}

}  // namespace at2v
