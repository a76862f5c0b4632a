// verify_host.cpp — TEST ONLY: compiles the product's device headers (at2-node_amd/csrc/*.h) for the
// host and checks verify_core against a golden fixture file. Never part of the shipped path.
// usage: verify_host <fixture.bin>   -> prints "n mismatches_dalek mismatches_sodium"
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include <map>

#include "at2v_comb.h"
#include "at2v_verify.h"
#include "at2v_verify_fu.h"
#include "at2v_fe_fu.h"

using namespace at2v;

struct HostTabA {
  ge_cached e[9];
  int pending = 0;
  void store(int i, const ge_cached& c) { e[i] = c; }
  void load(int i, ge_cached& c) const { c = e[i]; }
  void prefetch(int i) { pending = i; }
  void load_prefetched(ge_cached& c) const { c = e[pending]; }
};
struct HostTabB8 {
  void load(int i, ge_niels& n) const {
    const int32_t* p = &AT2V_BTAB[i * AT2V_BTAB_WORDS];
    for (int k = 0; k < 10; ++k) {
      n.ypx.v[k] = p[k];
      n.ymx.v[k] = p[10 + k];
      n.xy2d.v[k] = p[20 + k];
    }
  }
};
// [j]B, j = 0..2^15, built incrementally (P_j = P_{j-1} + B) and converted to affine Niels
struct HostTabB16 {
  std::vector<ge_niels> t;
  mutable int pending = 0;
  HostTabB16() {
    t.resize((1 << 15) + 1);
    ge_niels B1;
    HostTabB8().load(1, B1);
    ge_p3 P;
    ge_p3_identity(P);
    for (size_t j = 0; j < t.size(); ++j) {
      ge_p2 q;
      ge_p3_to_p2(q, P);
      ge_p2_to_niels(t[j], q);
      ge_p1p1 r;
      ge_madd(r, P, B1);
      ge_p1p1_to_p3(P, r);
    }
  }
  void prefetch(int e) const { pending = e; }
  void load_prefetched(ge_niels& n) const { n = t[pending]; }
};

// [j 2^128]B, j = 0..2^15, incrementally from the affine Niels form of [2^128]B
struct HostTabB16Hi {
  std::vector<ge_niels> t;
  mutable int pending = 0;
  HostTabB16Hi() {
    t.resize((1 << 15) + 1);
    const uint32_t s128[8] = {0, 0, 0, 0, 1, 0, 0, 0};
    ge_p2 Q;
    ge_scalarmult_base(Q, s128, HostTabB8());
    ge_niels N1;
    ge_p2_to_niels(N1, Q);
    ge_p3 P;
    ge_p3_identity(P);
    for (size_t j = 0; j < t.size(); ++j) {
      ge_p2 q;
      ge_p3_to_p2(q, P);
      ge_p2_to_niels(t[j], q);
      ge_p1p1 r;
      ge_madd(r, P, N1);
      ge_p1p1_to_p3(P, r);
    }
  }
  void prefetch(int e) const { pending = e; }
  void load_prefetched(ge_niels& n) const { n = t[pending]; }
};

struct HostTabAFu {
  gu_cached e[9];
  int pending = 0;
  void store(int i, const gu_cached& c) { e[i] = c; }
  gu_p3 parked;
  void park(const gu_p3& p) { parked = p; }
  void unpark(gu_p3& p) const { p = parked; }
  void prefetch(int i) { pending = i; }
  void load_prefetched(gu_cached& c) const { c = e[pending]; }
};
// unsigned-field copy of a signed-field fixed-base table
template <class T>
struct HostTabBFu {
  std::vector<gu_niels> t;
  mutable int pending = 0;
  explicit HostTabBFu(const T& src) {
    t.resize(src.t.size());
    for (size_t j = 0; j < t.size(); ++j) niels_fe_to_fu(t[j], src.t[j]);
  }
  void prefetch(int e) const { pending = e; }
  void load_prefetched(gu_niels& n) const { n = t[pending]; }
};

// comb of one key (at2v_comb.h), built by comb_build_lane over all lanes exactly as the device's builders do
struct HostComb {
  std::vector<uint32_t> w;  // kCombPos x kCombEntries entries of kCombWords words (the device's payload layout)
  int a_ok = 0;
  mutable int pend[2] = {0, 0};
  explicit HostComb(const uint32_t A[8]) : w((size_t)kCombPos * kCombEntries * kCombWords) {
    // keys alternate between the device's two builder shapes (8 and 2 lanes per position, at2v_comb.h)
    if (A[0] & 1) build<kCombWideLog2>(A);
    else build<kCombNarrowLog2>(A);
  }
  struct Mem {
    uint32_t* row;
    void put(int j, const uint32_t* src) const { std::memcpy(row + (size_t)j * kCombWords, src, kCombWords * 4); }
    void get(int j, uint32_t* dst) const { std::memcpy(dst, row + (size_t)j * kCombWords, kCombWords * 4); }
  };
  template <int kLog2>
  void build(const uint32_t A[8]) {
    for (int lane = 0; lane < (kCombPos << kLog2); ++lane) {
      const int pos = lane >> kLog2;
      Mem mem{w.data() + (size_t)(pos < kCombPos ? pos : 0) * kCombEntries * kCombWords};
      a_ok = comb_build_lane<kLog2>(A, pos, lane & ((1 << kLog2) - 1), mem);
    }
  }
  void prefetch(int st, int i, int j) const { pend[st] = i * kCombEntries + j; }
  void load_prefetched(int st, CombEntry& c) const {
    std::memcpy(&c, w.data() + (size_t)pend[st] * kCombWords, sizeof(CombEntry));
  }
};
// D[i][j] = [j 2^(W i)]B on demand (W = kBCombBits): (j 2^(16 i)) mod l times B by the signed-field base ladder, then the unsigned form
template <int W>
struct HostBCombW {
  static constexpr int kBits = W;
  mutable std::map<uint64_t, gu_niels> t;
  mutable uint64_t pend[2] = {0, 0};
  void prefetch(int st, int i, int j) const { pend[st] = ((uint64_t)i << 32) | (uint32_t)j; }
  void load_prefetched(int st, gu_niels& n) const {
    auto it = t.find(pend[st]);
    if (it == t.end()) {
      const int i = (int)(pend[st] >> 32);
      const uint32_t j = (uint32_t)pend[st];
      uint32_t x[16] = {0}, k[8];
      const int bit = W * i;
      x[bit >> 5] |= j << (bit & 31);
      if ((bit & 31) && (bit >> 5) + 1 < 16) x[(bit >> 5) + 1] |= (uint32_t)((uint64_t)j >> (32 - (bit & 31)));
      sc_reduce512(k, x);
      ge_p2 P;
      ge_scalarmult_base(P, k, HostTabB8());
      ge_niels ns;
      ge_p2_to_niels(ns, P);
      gu_niels nu;
      niels_fe_to_fu(nu, ns);
      it = t.emplace(pend[st], nu).first;
    }
    n = it->second;
  }
};

static void words(uint32_t w[8], const uint8_t* b) {
  for (int i = 0; i < 8; ++i) w[i] = (uint32_t)b[4 * i] | ((uint32_t)b[4 * i + 1] << 8) | ((uint32_t)b[4 * i + 2] << 16) | ((uint32_t)b[4 * i + 3] << 24);
}

int main(int argc, char** argv) {
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  uint32_t hdr[4];
  if (fread(hdr, 4, 4, f) != 4) return 2;
  size_t n = hdr[2], mb = hdr[3];
  std::vector<uint8_t> pk(32 * n), sig(64 * n), msg(mb + 8), vd(n), vs(n), cls(n);
  std::vector<uint32_t> off(n + 1);
  size_t ok = fread(pk.data(), 32, n, f) + fread(sig.data(), 64, n, f) + fread(off.data(), 4, n + 1, f);
  ok += fread(msg.data(), 1, mb, f) + fread(vd.data(), 1, n, f) + fread(vs.data(), 1, n, f) + fread(cls.data(), 1, n, f);
  fclose(f);
  (void)ok;
  size_t bad_d = 0, bad_s = 0;
  int limit = argc > 2 ? atoi(argv[2]) : (int)n;
  // 1: the half-size equation (verify_half); 2: on the unsigned field; 3: two lanes per signature (verify_pair_part);
  // 4: from per-key combs (verify_comb_fu, the sender-comb path); 5: the comb path's low-latency four-wave split;
  // 6: the four-wave kernel's split half-size check for chunks without combs (split_* in at2v_verify_fu.h)
  const int half = argc > 3 ? atoi(argv[3]) : 0;
  std::map<std::vector<uint32_t>, HostComb> combs;
  HostBCombW<kBCombBits> bcomb;        // verify_comb_fu (the throughput kernels' comb of B)
  HostBCombW<kBCombLatBits> bcomb_lat;  // the low-latency kernel's split forms (modes 5 and 6)
  for (size_t i = 0; i < n && (int)i < limit; ++i) {
    uint32_t R[8], A[8], S[8];
    words(R, &sig[64 * i]);
    words(S, &sig[64 * i + 32]);
    words(A, &pk[32 * i]);
    const uint8_t* m = &msg[off[i]];
    uint32_t len = off[i + 1] - off[i];
    auto mw = [&](uint32_t j) -> uint32_t {
      uint32_t v = 0;
      for (int b = 0; b < 4; ++b) if (4 * j + b < len) v |= (uint32_t)m[4 * j + b] << (8 * b);
      return v;
    };
    static HostTabB16 tb;
    HostTabA ta, tr;
    int d, s;
    if (half == 6) {  // wave 0 | wave 1 | wave 2, then the two ladders, -[t]B from the comb of B, and the combine
      auto split = [&](int policy) {
        HostTabAFu fa, fr;
        gu_p3 Ad, P0, P1;
        const int ok0 = split_a_side(Ad, R, A, S, policy, fa);
        const int ok1 = split_r_side(R, fr);
        uint32_t c0d[8], c1d[8], td[kBCombLatDigitWords];
        int c1_neg, nw;
        const int ok2 = split_scalars(c0d, c1d, td, c1_neg, nw, R, A, S, len, mw);
        nw = nw < 1 ? 1 : nw;  // (the kernel takes the wave maximum; one lane here)
        split_side_ladder(P0, c0d, nw, 0, fa);
        split_side_ladder(P1, c1d, nw, c1_neg, fr);
        gu_cached c1, ntb;
        gu_p3_to_cached(c1, P1);
        split_neg_tb(ntb, td, bcomb_lat);
        return ok0 & ok1 & ok2 & split_combine(P0, c1, ntb);
      };
      d = split(POLICY_DALEK_V1);
      s = split(POLICY_LIBSODIUM_1_0_18);
    } else if (half == 5) {  // the low-latency kernel's four-way split (comb_decode_r | B sum | A sums) and comb_check_split
      std::vector<uint32_t> key(A, A + 8);
      auto it = combs.find(key);
      if (it == combs.end()) it = combs.try_emplace(key, A).first;
      const HostComb& c = it->second;
      auto split = [&](int policy) {
        gu_p3 Rp, Pb, Pa0, Pa1;
        const int ok0 = comb_decode_r(Rp, R) & comb_prechecks(R, A, S, policy, c.a_ok);
        uint32_t sd[kBCombLatDigitWords], kd[kCombDigitWords];
        bcomb_recode<kBCombLatBits>(sd, S);
        gu_p3_identity(Pb);
        comb_sum<false>(Pb, sd, 0, kBCombLatPos, bcomb_lat);
        comb_k_digits(kd, R, A, len, mw);
        gu_p3_identity(Pa0);
        gu_p3_identity(Pa1);
        comb_sum<true>(Pa0, kd, 0, kCombPos / 2, c);
        comb_sum<true>(Pa1, kd, kCombPos / 2, kCombPos, c);
        return ok0 & comb_check_split(Rp, Pa0, Pa1, Pb);
      };
      d = split(POLICY_DALEK_V1);
      s = split(POLICY_LIBSODIUM_1_0_18);
    } else if (half == 4) {
      std::vector<uint32_t> key(A, A + 8);
      auto it = combs.find(key);
      if (it == combs.end()) it = combs.try_emplace(key, A).first;
      const HostComb& c = it->second;
      d = verify_comb_fu(R, A, S, len, mw, POLICY_DALEK_V1, c.a_ok, c, bcomb);
      s = verify_comb_fu(R, A, S, len, mw, POLICY_LIBSODIUM_1_0_18, c.a_ok, c, bcomb);
    } else if (half == 3) {
      static HostTabB16Hi tb1s;
      static HostTabBFu<HostTabB16> fb0(tb);
      static HostTabBFu<HostTabB16Hi> fb1(tb1s);
      auto one = [](int v) { return v; };
      auto pair = [&](int policy) {
        HostTabAFu f0, f1;
        gu_p3 P0, P1;
        const int ok0 = verify_pair_part(0, R, A, S, len, mw, policy, f0, fb0, one, P0);
        const int ok1 = verify_pair_part(1, R, A, S, len, mw, policy, f1, fb1, one, P1);
        gu_cached c1;
        gu_p3_to_cached(c1, P1);
        return ok0 & ok1 & verify_pair_combine(P0, c1);
      };
      d = pair(POLICY_DALEK_V1);
      s = pair(POLICY_LIBSODIUM_1_0_18);
    } else if (half == 2) {
      static HostTabB16Hi tb1s;
      static HostTabBFu<HostTabB16> fb0(tb);
      static HostTabBFu<HostTabB16Hi> fb1(tb1s);
      HostTabAFu fa, fr;
      auto one = [](int v) { return v; };
      d = verify_half_fu(R, A, S, len, mw, POLICY_DALEK_V1, fa, fr, fb0, fb1, one);
      s = verify_half_fu(R, A, S, len, mw, POLICY_LIBSODIUM_1_0_18, fa, fr, fb0, fb1, one);
    } else if (half) {
      static HostTabB16Hi tb1;
      auto one = [](int v) { return v; };
      d = verify_half(R, A, S, len, mw, POLICY_DALEK_V1, ta, tr, tb, tb1, one);
      s = verify_half(R, A, S, len, mw, POLICY_LIBSODIUM_1_0_18, ta, tr, tb, tb1, one);
    } else {
      auto rl = [&](uint32_t r[8]) { for (int q = 0; q < 8; ++q) r[q] = R[q]; };
      d = verify_core<16>(R, A, S, len, mw, POLICY_DALEK_V1, ta, tb, rl);
      s = verify_core<16>(R, A, S, len, mw, POLICY_LIBSODIUM_1_0_18, ta, tb, rl);
    }
    if (d != vd[i]) { if (bad_d < 10) fprintf(stderr, "dalek mismatch i=%zu cls=%d got=%d want=%d\n", i, cls[i], d, vd[i]); ++bad_d; }
    if (s != vs[i]) { if (bad_s < 10) fprintf(stderr, "sodium mismatch i=%zu cls=%d got=%d want=%d\n", i, cls[i], s, vs[i]); ++bad_s; }
  }
  printf("%zu %zu %zu\n", n, bad_d, bad_s);
  return (bad_d || bad_s) ? 1 : 0;
}
