// at2v_kernels.hip — gfx950 kernels: batch verify (the hot path) and the GPU record generator / signer.
//
// Verify kernel layout (the full-length form of §4 is the AT2V_VERIFY_HALF=0 build):
//   * one lane = one signature; a wave owns a contiguous chunk of 64 records, so the verdict bits of a
//     chunk are one __ballot -> two uint32 words written by lane 0 (no atomics, no cross-wave traffic);
//   * persistent grid (resident waves only), chunks c = wave_id + k * total_waves; each wave reuses a
//     fixed 180 KiB slice of the scratch buffer for its 64 lanes' tables [0..8]A and [0..8](+-R) (cached
//     form, 160 B per entry, lane-contiguous);
//   * the fixed-base tables [0..2^15]B and [0..2^15] 2^128 B (affine Niels, 128 B per entry, 8.4 MB) are
//     built once per context and stay L2/MALL-resident; table entries reach the lanes by LDS-DMA;
//   * records are read straight from the ABI layout (pk n x 32, sig n x 64, msg + offsets) with
//     16-byte loads for A/R/S and 4-byte loads + v_alignbit for unaligned message words.
#include <hip/hip_runtime.h>

#include "../../include/at2v.h"
#include "at2v_cache.h"
#include "at2v_comb.h"
#include "at2v_verify.h"
#include "at2v_verify_fu.h"
#include "at2v_fe_fu.h"

namespace at2v {

#ifndef AT2V_FIELD_FU
#define AT2V_FIELD_FU 1  // 1: verify on the unsigned chained-carry field; 0: balanced signed field (§3)
#endif

#ifndef AT2V_VERIFY_WAVES_PER_SIMD
#define AT2V_VERIFY_WAVES_PER_SIMD 2  // register budget: 512 / waves VGPR+AGPR per lane
#endif

#ifndef AT2V_VERIFY_HALF
#define AT2V_VERIFY_HALF 1  // 1: half-size equation; 0: full-length ladder (§4)
#endif
#ifndef AT2V_BWIN
#define AT2V_BWIN 16  // fixed-base window bits: table [0..2^(AT2V_BWIN-1)]B
#endif
#if AT2V_VERIFY_HALF && AT2V_BWIN != 16
#error "the half-size path uses 16-bit fixed-base windows"
#endif
#ifndef AT2V_LADDER_BW
#define AT2V_LADDER_BW 16  // fixed-base window of the throughput ladder kernels (verify_half_fu kBW); 24: two shared 1 GB
                           // tables, 12 B additions instead of 16: +0.1% (106.05 vs 105.92 M/s, profiles/r06/r06l), not adopted
#endif
#ifndef AT2V_INV_GROUP
#define AT2V_INV_GROUP 2  // chunks whose final inversions share one field inversion (Montgomery's trick)
#endif

#ifndef AT2V_BLOCK
#define AT2V_BLOCK 512  // verify threads per block: 8 waves, both waves of every SIMD in one workgroup
#endif
#ifndef AT2V_QUEUE
#define AT2V_QUEUE 1  // 1: chunks after the first come from the per-launch queue; 0: static c += nwaves
#endif
#ifndef AT2V_SOLO_TAIL
#define AT2V_SOLO_TAIL 0  // 1: waves 4..7 stop pulling chunks for the last nwaves/2 chunks of a launch
#endif
#ifndef AT2V_FAIR
#define AT2V_FAIR 1  // 1: the two waves of a SIMD pace each other with s_setprio (needs AT2V_BLOCK 512)
#endif
constexpr int kBlock = AT2V_BLOCK;
constexpr int kWavesPerBlock = kBlock / 64;
static_assert(!AT2V_FAIR || kBlock == 512, "pacing pairs waves w and w^4 of an 8-wave workgroup");
// control words after the lane slots of a launch's `grid` blocks: [0] chunk queue counter; from word 16 on,
// one 64-byte progress line per wave (AT2V_FAIR)
constexpr size_t kCtlBytes(int grid) { return 64 + (size_t)grid * kWavesPerBlock * 64; }
constexpr int kBWin = AT2V_BWIN;
constexpr int kGroup = AT2V_INV_GROUP;
static_assert(kGroup >= 1 && kGroup <= 8, "inversion group");
// AT2V_IDENT_SHARED (half-size path): entry 0 of every per-lane table is the identity, so it is not stored per lane:
// a digit 0 reads one shared, L2-resident identity entry after the B tables instead. Per-lane tables hold [1..8]P
// (1280 B instead of 1440 B: 11% less table footprint and write traffic, 1/16 of the entry reads served from L2).
#ifndef AT2V_IDENT_SHARED
#define AT2V_IDENT_SHARED AT2V_VERIFY_HALF
#endif
constexpr int kIdentShared = AT2V_IDENT_SHARED ? 1 : 0;
constexpr int kTabAGranules = (9 - kIdentShared) * 10;  // entries (1 or 0)..8 x 10 x 16 B
#if AT2V_VERIFY_HALF
constexpr int kLaneGranules = 2 * kTabAGranules;  // tables [j]A and [j](+-R)
constexpr int kNumBtabs = 2;                      // [j]B and [j 2^128]B
#else
constexpr int kParkGranules = 8 * kGroup;        // parked R' (X, Y, Z: 30 words) of every chunk of a group
constexpr int kPrefGranules = 3 * (kGroup - 1);  // prefix products Z_0..Z_h of the group (10 words each)
constexpr int kLaneGranules = kTabAGranules + kParkGranules + kPrefGranules;
constexpr int kNumBtabs = 1;
#endif
constexpr size_t kScratchPerWave = (size_t)kLaneGranules * 64 * 16;
#ifndef AT2V_EXP_COMB3
#define AT2V_EXP_COMB3 0  // EXPERIMENT ONLY (wrong verdicts): the hit-list comb kernel in 768-thread blocks at three waves per
                          // SIMD (<= 168 VGPRs), each wave's two LDS stages aliased onto one 10 KB region (VERDICT r5 "Next" 5)
#endif
constexpr int kWavesAlloc = AT2V_EXP_COMB3 ? 12 : kWavesPerBlock;  // lane-slot sets per block of the scratch buffer

// A value the compiler cannot prove wave-uniform but that is (the wave index in the block): as an SGPR, the LDS-DMA
// destinations (M0) need no v_readfirstlane per load. AT2V_WIB_UNIFORM=0: plain VGPR (A/B).
#ifndef AT2V_WIB_UNIFORM
#define AT2V_WIB_UNIFORM 1
#endif
#if AT2V_WIB_UNIFORM
#define AT2V_UNIFORM(x) __builtin_amdgcn_readfirstlane(x)
#else
#define AT2V_UNIFORM(x) (x)
#endif

// Per-lane table [0..8](-A) in global scratch. Layout: lane-contiguous, 9 entries x 160 B per lane
// (1440 B), so the 10 16-byte loads of one entry hit the same 2 cache lines per lane (L1-resident
// across the 10 loads) whatever entry index each lane selects. (r01 interleaved lanes per 16-byte
// granule: lanes with different digits then touched up to 9 different 1 KiB rows per load,
// ~9x read amplification — profiles/r01 FETCH_SIZE.)
// AT2V_TAB_PACK = 1: per-lane table entries packed into 128 B, one cache line per entry instead of two (the table reads
// of a verify go from ~16.9 to ~8.4 KB). Each coordinate is carried at the table build and its 10 limbs
// (255 bits, limb 1 given a 26th bit for its carry) packed into 8 words: word k holds limb k (k < 8) in its low 26 or
// 25 bits, and limbs 8 and 9 (51 bits) fill the words' free high bits. A timing-only build with the entries truncated
// to one line measured +3.6% (AT2V_EXP_TAB128, profiles/r04zi); with the carries and the unpacking, +1.0% and +0.1%
// (medians; minima +0.6%, +0.8%) in two A/B runs, GPU suite 103 passed on it (profiles/r04zk). Default since round 4.
#ifndef AT2V_TAB_PACK
#define AT2V_TAB_PACK 1
#endif

// carried element -> 8 words (see AT2V_TAB_PACK)
__device__ AT2V_INLINE void fu_pack8(uint32_t o[8], const fu& f) {
  const uint32_t hl = f.v[8] | (f.v[9] << 26), hh = f.v[9] >> 6;  // H = limb 8 | limb 9 << 26 (51 bits)
  o[0] = f.v[0] | (hl << 26);
  o[1] = f.v[1] | ((hl >> 6) << 26);
  o[2] = f.v[2] | ((hl >> 12) << 26);
  o[3] = f.v[3] | ((hl >> 18) << 25);
  o[4] = f.v[4] | ((hl >> 25) << 26);
  o[5] = f.v[5] | (((hl >> 31) | (hh << 1)) << 25);
  o[6] = f.v[6] | ((hh >> 6) << 26);
  o[7] = f.v[7] | ((hh >> 12) << 25);
}
__device__ AT2V_INLINE void fu_unpack8(fu& f, const uint32_t i[8]) {
  const uint32_t m26 = (1u << 26) - 1, m25 = (1u << 25) - 1;
  f.v[0] = i[0] & m26;
  f.v[1] = i[1] & m26;
  f.v[2] = i[2] & m26;
  f.v[3] = i[3] & m25;
  f.v[4] = i[4] & m26;
  f.v[5] = i[5] & m25;
  f.v[6] = i[6] & m26;
  f.v[7] = i[7] & m25;
  const uint32_t p5 = i[5] >> 25;
  const uint32_t hl = (i[0] >> 26) | ((i[1] >> 26) << 6) | ((i[2] >> 26) << 12) | ((i[3] >> 25) << 18) |
                      ((i[4] >> 26) << 25) | (p5 << 31);
  const uint32_t hh = (p5 >> 1) | ((i[6] >> 26) << 6) | ((i[7] >> 25) << 12);
  f.v[8] = hl & m26;
  f.v[9] = ((hl >> 26) | (hh << 6)) & m25;
}

struct DevTabA {
  int4* base;   // this lane's slot (global): entries kIdentShared..8, 160 B each (128 B with AT2V_TAB_PACK)
  int4* stage;  // this wave's 10 x 1 KiB LDS staging buffer for the prefetched entry
  int lane;
  const int4* ident = nullptr;  // the shared identity entry (kIdentShared)
#ifdef AT2V_WAIT_PROBE
  mutable unsigned long long waited = 0, lds_waited = 0;
#endif
  template <class Cached>
  __device__ AT2V_INLINE void store(int e, const Cached& c) const {
    static_assert(sizeof(Cached) == 160, "cached point: 40 words");
    if (kIdentShared && e == 0) return;  // the identity lives in the shared entry
    const int32_t* w = reinterpret_cast<const int32_t*>(&c);
#if AT2V_TAB_PACK
    {
      uint32_t pw[32];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        fu x;
#pragma unroll
        for (int q = 0; q < 10; ++q) x.v[q] = (uint32_t)w[10 * k + q];
        fu_carry(x);
        fu_pack8(pw + 8 * k, x);
      }
#pragma unroll
      for (int q = 0; q < 8; ++q)
        base[(e - kIdentShared) * 8 + q] =
            make_int4((int)pw[4 * q], (int)pw[4 * q + 1], (int)pw[4 * q + 2], (int)pw[4 * q + 3]);
      return;
    }
#endif
#if AT2V_EXP_TAB128  // EXPERIMENT (wrong verdicts, timing only): 128-byte entries, one line each (the last 8 words dropped)
#pragma unroll
    for (int q = 0; q < 8; ++q)
      base[(e - kIdentShared) * 8 + q] = make_int4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
    return;
#endif
#pragma unroll
    for (int q = 0; q < 10; ++q)
      base[(e - kIdentShared) * 10 + q] = make_int4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
  }
  // a decoded point parked in entry 8's space (verify_half_fu, AT2V_PARK_POINTS): 10 stores now, 10 loads and one wait
  // at unpark; entry 8 is the last one the table build writes
  template <class P3>
  __device__ AT2V_INLINE void park(const P3& p) const {
    static_assert(sizeof(P3) == 160, "p3 point: 40 words");
    const int32_t* w = reinterpret_cast<const int32_t*>(&p);
#pragma unroll
    for (int q = 0; q < 10; ++q)
      base[(8 - kIdentShared) * 10 + q] = make_int4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
  }
  template <class P3>
  __device__ AT2V_INLINE void unpark(P3& p) const {
    int32_t* w = reinterpret_cast<int32_t*>(&p);
    int4 v[10];
#pragma unroll
    for (int q = 0; q < 10; ++q) v[q] = base[(8 - kIdentShared) * 10 + q];
#pragma unroll
    for (int q = 0; q < 10; ++q) {
      w[4 * q] = v[q].x;
      w[4 * q + 1] = v[q].y;
      w[4 * q + 2] = v[q].z;
      w[4 * q + 3] = v[q].w;
    }
  }
  __device__ AT2V_INLINE void load(int e, ge_cached& c) const {
    int32_t* w = reinterpret_cast<int32_t*>(&c);
#pragma unroll
    for (int q = 0; q < 10; ++q) {
      const int4 v = base[e * 10 + q];
      w[4 * q] = v.x;
      w[4 * q + 1] = v.y;
      w[4 * q + 2] = v.z;
      w[4 * q + 3] = v.w;
    }
  }
  // LDS-DMA (global_load_lds_dwordx4): entry e of every lane -> stage[q][lane], no VGPRs held while the
  // window's four doublings run
  __device__ AT2V_INLINE void prefetch(int e) const {
#if AT2V_EXP_TAB128 || AT2V_TAB_PACK
    const int4* src = (kIdentShared && e == 0) ? ident : base + (e - kIdentShared) * 8;
#pragma unroll
    for (int q = 0; q < 8; ++q)
#else
    const int4* src = (kIdentShared && e == 0) ? ident : base + (e - kIdentShared) * 10;
#pragma unroll
    for (int q = 0; q < 10; ++q)
#endif
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src + q),
                                       (__attribute__((address_space(3))) void*)(stage + q * 64), 16,
                                       0, 0);
  }
  template <class Cached>
  __device__ AT2V_INLINE void load_prefetched(Cached& c) const {
    static_assert(sizeof(Cached) == 160, "cached point: 40 words");
    AT2V_PROBE(waited, asm volatile("s_waitcnt vmcnt(0)" ::: "memory"));
    int32_t* w = reinterpret_cast<int32_t*>(&c);
#if AT2V_TAB_PACK
    {
      uint32_t pw[32];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int4 v = stage[q * 64 + lane];
        pw[4 * q] = (uint32_t)v.x;
        pw[4 * q + 1] = (uint32_t)v.y;
        pw[4 * q + 2] = (uint32_t)v.z;
        pw[4 * q + 3] = (uint32_t)v.w;
      }
      fu* cf = reinterpret_cast<fu*>(&c);
#pragma unroll
      for (int k = 0; k < 4; ++k) fu_unpack8(cf[k], pw + 8 * k);
      return;
    }
#endif
#pragma unroll
    for (int q = 0; q < 10; ++q) {
      const int4 v = stage[q * 64 + lane];
      w[4 * q] = v.x;
      w[4 * q + 1] = v.y;
      w[4 * q + 2] = v.z;
      w[4 * q + 3] = v.w;
    }
#ifdef AT2V_WAIT_PROBE
    AT2V_PROBE(lds_waited, asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"));
#endif
  }
};

struct LdsTabB {
  const int4* lds;  // AT2V_BTAB_ENTRIES x 8 granules
  __device__ AT2V_INLINE void load(int e, ge_niels& n) const {
    int32_t w[32];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int4 v = lds[e * 8 + q];
      w[4 * q] = v.x;
      w[4 * q + 1] = v.y;
      w[4 * q + 2] = v.z;
      w[4 * q + 3] = v.w;
    }
#pragma unroll
    for (int k = 0; k < 10; ++k) {
      n.ypx.v[k] = w[k];
      n.ymx.v[k] = w[10 + k];
      n.xy2d.v[k] = w[20 + k];
    }
  }
};

// Fixed-base table [0..2^(kBWin-1)]B (affine Niels, 8 x 16 B per entry: 4.2 MB for 16-bit windows,
// 67 MB for 20, 1.07 GB for 24) in global memory, read through an LDS-DMA prefetch like the A entries.
constexpr int kBtabEntries = (1 << (kBWin - 1)) + 1;
constexpr int kLadderEntries = (1 << 23) + 1;  // entries of each 24-bit ladder table (AT2V_LADDER_BW 24)
struct DevTabB {
  const int4* base;
  int4* stage;  // this wave's 8 x 1 KiB LDS staging buffer
  int lane;
#ifdef AT2V_WAIT_PROBE
  mutable unsigned long long waited = 0, lds_waited = 0;
#endif
  __device__ AT2V_INLINE void prefetch(int e) const {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the stage may be shared with a just-read entry
#pragma unroll
    for (int q = 0; q < 8; ++q)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(base + e * 8 + q),
                                       (__attribute__((address_space(3))) void*)(stage + q * 64), 16, 0, 0);
  }
  template <class Niels>
  __device__ AT2V_INLINE void load_prefetched(Niels& n) const {
    static_assert(sizeof(Niels) == 120, "Niels point: 30 words");
    AT2V_PROBE(waited, asm volatile("s_waitcnt vmcnt(0)" ::: "memory"));
    int32_t w[32];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int4 v = stage[q * 64 + lane];
      w[4 * q] = v.x;
      w[4 * q + 1] = v.y;
      w[4 * q + 2] = v.z;
      w[4 * q + 3] = v.w;
    }
#pragma unroll
    for (int k = 0; k < 10; ++k) {
      n.ypx.v[k] = w[k];
      n.ymx.v[k] = w[10 + k];
      n.xy2d.v[k] = w[20 + k];
    }
  }
};

// Per-wait probe of the comb kernel (a variant build: tools/build_variant.sh <tag> -DAT2V_COMB_PROBE, read by
// tools/ab_bench.py --probe through at2v_probe_read): s_memtime cycles per wave in each wait and phase of
// verify_chunks_comb4, summed over the launch. Product builds: just stmt.
#if defined(AT2V_COMB_PROBE) && defined(__HIP_DEVICE_COMPILE__)
#define AT2V_CPROBE(acc, stmt)                                  \
  do {                                                          \
    const unsigned long long t0_ = __builtin_amdgcn_s_memtime(); \
    stmt;                                                       \
    (acc) += __builtin_amdgcn_s_memtime() - t0_;                \
  } while (0)
#else
#define AT2V_CPROBE(acc, stmt) stmt
#endif
#ifdef AT2V_COMB_PROBE
enum {
  kCpAWait,     // A-comb entry: vmcnt wait before the stage is read
  kCpBWait,     // B-comb entry: the same
  kCpStage,     // lgkmcnt wait before a stage is refilled
  kCpRecord,    // the record's R, S, A, offsets loaded + the prechecks
  kCpSha,       // SHA-512(R || A || M) mod l, recodes (message loads included)
  kCpSums,      // the 26 A + 16 B comb additions (the three waits above included)
  kCpFinish,    // slot round trip, shared inversion, four encodes + compares
  kCpBook,      // list loads, verdict ORs, chunk ticket
  kCpChunk,     // chunk total
  kCpChunks,    // chunks (count)
  kCpLds,       // comb entries: lgkmcnt wait after the stage's LDS reads (forced in the probe build)
  kCpSlot,      // parked points: vmcnt wait after the slot loads of the inversion and encodes (forced likewise)
  kCpN
};
__device__ unsigned long long at2v_cprobe_acc[kCpN];
struct CombProbe {
  unsigned long long v[kCpN] = {};
};
#endif

// Comb entries (at2v_comb.h) by LDS-DMA into two alternating per-wave stages: the entry of the next addition lands while
// this one is computed. TabC: C[i][j] of this lane's key (CombEntry, kCombGranules); TabBC: D[i][j] (affine Niels, 8).
struct DevComb {
  const int4* base;  // this lane's key's comb
  int4* stage[2];    // this wave's two 10 KiB stages (wave-uniform)
  int lane;
#ifdef AT2V_COMB_PROBE
  mutable unsigned long long waited = 0, stage_waited = 0, lds_waited = 0;
#endif
  __device__ AT2V_INLINE void prefetch(int st, int i, int j) const {
    AT2V_CPROBE(stage_waited, asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"));  // the stage's previous entry is read
#if AT2V_EXP_COMB_HOT  // EXPERIMENT (wrong verdicts, timing only): every A entry read is the same cache-hot line
    i = 0;
    j = 1;
#endif
    const int4* src = base + ((size_t)i * kCombEntries + j) * kCombGranules;
#pragma unroll
    for (int q = 0; q < kCombGranules; ++q)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src + q),
                                       (__attribute__((address_space(3))) void*)(stage[st] + q * 64), 16, 0, 0);
  }
  __device__ AT2V_INLINE void load_prefetched(int st, CombEntry& c) const {
    static_assert(sizeof(CombEntry) <= (size_t)kCombWords * 4, "comb entry words");
    AT2V_CPROBE(waited, asm volatile("s_waitcnt vmcnt(0)" ::: "memory"));
    int32_t w[kCombWords];
#pragma unroll
    for (int q = 0; q < kCombGranules; ++q) {
      const int4 v = stage[st][q * 64 + lane];
      w[4 * q] = v.x;
      w[4 * q + 1] = v.y;
      w[4 * q + 2] = v.z;
      w[4 * q + 3] = v.w;
    }
#ifdef AT2V_COMB_PROBE
    AT2V_CPROBE(lds_waited, asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"));
#endif
    int32_t* cw = reinterpret_cast<int32_t*>(&c);
#pragma unroll
    for (int q = 0; q < (int)(sizeof(CombEntry) / 4); ++q) cw[q] = w[q];
  }
};
template <int W>
struct DevBCombW {
  static constexpr int kBits = W;
  const int4* base;  // the context's comb of B (W-bit windows)
  int4* stage[2];
  int lane;
#ifdef AT2V_COMB_PROBE
  mutable unsigned long long waited = 0, stage_waited = 0, lds_waited = 0;
#endif
  __device__ AT2V_INLINE void prefetch(int st, int i, int j) const {
    AT2V_CPROBE(stage_waited, asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"));
#if AT2V_EXP_COMB_HOT
    i = 0;
    j = 1;
#endif
    const int4* src = base + ((size_t)i * BCombGeom<W>::kEntries + j) * 8;
#pragma unroll
    for (int q = 0; q < 8; ++q)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src + q),
                                       (__attribute__((address_space(3))) void*)(stage[st] + q * 64), 16, 0, 0);
  }
  template <class Niels>
  __device__ AT2V_INLINE void load_prefetched(int st, Niels& n) const {
    static_assert(sizeof(Niels) == 120, "Niels point: 30 words");
    AT2V_CPROBE(waited, asm volatile("s_waitcnt vmcnt(0)" ::: "memory"));
    int32_t w[32];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int4 v = stage[st][q * 64 + lane];
      w[4 * q] = v.x;
      w[4 * q + 1] = v.y;
      w[4 * q + 2] = v.z;
      w[4 * q + 3] = v.w;
    }
#ifdef AT2V_COMB_PROBE
    AT2V_CPROBE(lds_waited, asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"));
#endif
#pragma unroll
    for (int k = 0; k < 10; ++k) {
      n.ypx.v[k] = w[k];
      n.ymx.v[k] = w[10 + k];
      n.xy2d.v[k] = w[20 + k];
    }
  }
};
using DevBCombLat = DevBCombW<kBCombLatBits>;  // every context with combs (all other comb paths)

__device__ AT2V_INLINE void stage_btab(int4* lds) {
  const int4* src = reinterpret_cast<const int4*>(AT2V_BTAB);
  for (int i = threadIdx.x; i < AT2V_BTAB_ENTRIES * 8; i += blockDim.x) lds[i] = src[i];
  __syncthreads();
}

__device__ AT2V_INLINE void load8(uint32_t w[8], const uint8_t* p) {  // 32 bytes, 16-B aligned
  const uint4 a = reinterpret_cast<const uint4*>(p)[0];
  const uint4 b = reinterpret_cast<const uint4*>(p)[1];
  w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
  w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
}

// little-endian 32-bit word at byte address a of a buffer of `total` bytes; bytes >= total read as 0
__device__ AT2V_INLINE uint32_t load_u32_guarded(const uint8_t* buf, uint32_t a, uint32_t total) {
  if (a + 4 <= total) return *reinterpret_cast<const uint32_t*>(buf + a);
  uint32_t v = 0;
  for (uint32_t b = 0; b < 4; ++b)
    if (a + b < total) v |= (uint32_t)buf[a + b] << (8 * b);
  return v;
}

// store / load a group-local field element or p2 point in this lane's scratch slot (lane-contiguous)
__device__ AT2V_INLINE void slot_store(int4* dst, const int32_t* w, int nw) {
  for (int q = 0; q < (nw + 3) / 4; ++q)
    dst[q] = make_int4(w[4 * q], 4 * q + 1 < nw ? w[4 * q + 1] : 0, 4 * q + 2 < nw ? w[4 * q + 2] : 0,
                       4 * q + 3 < nw ? w[4 * q + 3] : 0);
}
__device__ AT2V_INLINE void slot_load(int32_t* w, const int4* src, int nw) {
  for (int q = 0; q < (nw + 3) / 4; ++q) {
    const int4 v = src[q];
    w[4 * q] = v.x;
    if (4 * q + 1 < nw) w[4 * q + 1] = v.y;
    if (4 * q + 2 < nw) w[4 * q + 2] = v.z;
    if (4 * q + 3 < nw) w[4 * q + 3] = v.w;
  }
}

#if AT2V_VERIFY_HALF
__device__ AT2V_INLINE int wave_max_i32(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int u = __shfl_xor(v, o);
    v = u > v ? u : v;
  }
  return __builtin_amdgcn_readfirstlane(v);
}

#if AT2V_FAIR
// Pacing of the two waves that share a SIMD (an 8-wave workgroup places waves w and w^4 on one SIMD;
// MI355X guide, "Two waves per SIMD"). VALU issue goes by priority, then age, so without it the older wave
// runs nearly unimpeded and the younger gets leftover slots. Each wave publishes its progress (work units,
// ~1 per ladder window) and raises its priority while it trails its partner. The partner's value is read
// one mark late (the load issued at mark k is consumed at mark k+1), so the loads' latency is hidden; a
// stale value only misjudges one interval. Stores are vector stores from lane 0.
#ifndef AT2V_FAIR_LAG
#define AT2V_FAIR_LAG -1  // >= 0: half-window progress units, the younger half trails its partner by this many
#endif
struct Pace {
  uint32_t* mine;
  const uint32_t* mate;
  uint32_t prog;
  uint32_t mate_prog;
  int lag;  // 0 for waves 0..3; AT2V_FAIR_LAG for waves 4..7 (their target lead is negative)
#ifdef AT2V_WAIT_PROBE
  unsigned long long probe[4] = {0, 0, 0, 0};  // digit reads, mid-window mark, chunk total, chunk-start loads
#endif
#if AT2V_FAIR_LAG >= 0
  __device__ AT2V_INLINE void mark(uint32_t units) { step(2 * units); }
  __device__ AT2V_INLINE void window() { step(1); }
  __device__ AT2V_INLINE void mid() { step(1); }
#else
  __device__ AT2V_INLINE void mark(uint32_t units) { step(units); }
  __device__ AT2V_INLINE void window() { step(1); }
  __device__ AT2V_INLINE void mid() {}
#endif
  __device__ AT2V_INLINE void step(uint32_t units) {
    prog += units;
    const uint32_t behind = __builtin_amdgcn_readfirstlane((int)(mate_prog - prog) > lag ? 1u : 0u);
    if (behind) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
    if ((threadIdx.x & 63) == 0) __hip_atomic_store(mine, prog, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    mate_prog = __hip_atomic_load(mate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
};
#endif

// ---- per-sender A cache (at2v_opts.sender_cache; at2v_cache.h) ----
// An entry (4 granules, one 64-byte line): key = the 32 bytes of A, meta = {dalek decode verdict of A, valid, payload
// index u (-1: none), epoch of the last launch that used it}. A fingerprint only nominates an entry: a record takes it
// only if it is valid (its payload built and flipped by an earlier launch's build stream) and all 32 key bytes equal the
// record's A, so a collision, a claim without a payload or an entry still being built costs speed, never a verdict.
// Plain loads of an entry may be stale across XCDs inside one launch; every stale state (valid = 0, a zero key) only
// turns a hit into a miss, because an entry's key never changes while its tag table is live and valid only goes 0 -> 1.
constexpr int kCacheEntryGranules = 4;
constexpr int kCtlWords = kCtlWordsTotal;

__device__ AT2V_INLINE uint64_t cache_fingerprint(const uint32_t a[8], uint64_t seed, uint64_t mask) {
  uint64_t h = seed;
#pragma unroll
  for (int i = 0; i < 8; i += 2) {
    h ^= (uint64_t)a[i] | ((uint64_t)a[i + 1] << 32);
    h *= 0x9e3779b97f4a7c15ull;
    h ^= h >> 29;
  }
  h *= 0xbf58476d1ce4e5b9ull;
  h ^= h >> 32;
  return (h & mask) | 1ull;  // never 0 (= free)
}

// One record per lane, called by every lane of a wave (ballots): find A's entry by fingerprint (open addressing, 32
// probes) or claim a free tag (64-bit CAS). Lanes of the wave that want the same new key elect one leader (the lowest
// lane), which claims for all of them. A claim takes a payload index from the free list (one atomic per wave) and writes
// the entry's key and meta {0, valid 0, u, epoch}; claims that got a payload are appended to the launch's claim set for
// the build stream. A claim that finds the free list empty (u = -1) or a record whose probe path is full flags the cache
// full (compaction before the next launch). Returns the entry slot or -1.
// statistics of a caller that sums its lookups itself (wave-uniform), instead of one atomic per counter per wave
struct LookupStats {
  uint32_t found = 0, claimed = 0, failed = 0, sighted = 0;
};

__device__ AT2V_INLINE int cache_lookup_wave(const CacheArgs& c, const uint32_t a[8], int lane, bool active = true,
                                             LookupStats* st = nullptr) {
  const uint32_t mask = c.cap - 1;
  int slot = -1, claimed = 0, found = 0, want = 0;
  uint64_t fp = cache_fingerprint(a, c.seed, c.fp_mask);
  uint32_t h = (uint32_t)(fp >> 17) & mask, k = 0;
  for (; k < 32; ++k) {  // phase 1: find the key, or the first free tag on its probe path
    const unsigned long long t =
        __hip_atomic_load(c.tags + ((h + k) & mask), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == fp) {
      slot = (int)((h + k) & mask);
      found = 1;
      break;
    }
    if (t == 0) {
      want = 1;
      break;
    }
  }
  // a lane past the end of the batch (it recomputes the last record) looks up but neither claims nor counts as a sighting
  if (!active) want = 0;
  // a lane whose key is deferred (no claims while a compaction runs, or a first sighting) is a plain miss, not a failure
  int deferred = 0;
  if (c.no_claim && want) {  // a compaction is running: look up only (the records of a new key are misses)
    want = 0;
    deferred = 1;
  }
  int leader = lane, nsame = 0;
  {
    uint64_t pending = __ballot(want);
    while (pending) {  // one iteration per distinct wanted key in the wave
      const int L = __ffsll((long long)pending) - 1;
      const uint64_t fpL = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(fp >> 32), L) << 32) |
                           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)fp, L);
      const int same = want && fp == fpL;
      const uint64_t sm = __ballot(same);
      if (same) {
        leader = L;
        nsame = __popcll(sm);
      }
      pending &= ~sm;
    }
  }
  const int follower = want && leader != lane;
  // admission: the wave's leader of a new key claims it only at its second sighting (or with 2+ records in this wave)
  int sighted = 0;
  if (want && !follower && !c.admit_first && nsame < 2) {
    unsigned long long* sp = c.seen + ((uint32_t)(fp >> 40) & c.seen_mask);
    if (__hip_atomic_load(sp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != fp) {
      __hip_atomic_store(sp, (unsigned long long)fp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      sighted = 1;
    }
  }
  {
    const int ls = __shfl(sighted, leader);  // (every lane takes part in the shuffle)
    if (want && ls) deferred = 1;
  }
  if (want && !follower && !sighted) {  // phase 2: claim along the probe path (a racing claimant may take the tag first)
    for (; k < 32; ++k) {
      const uint32_t j = (h + k) & mask;
      const unsigned long long old = atomicCAS(c.tags + j, 0ull, (unsigned long long)fp);
      if (old == 0) {
        slot = (int)j;
        claimed = 1;
        break;
      }
      if (old == fp) {
        slot = (int)j;
        found = 1;
        break;
      }
    }
  }
  {  // followers take their leader's outcome (a shuffle: every lane of the wave takes part)
    const int ls = __shfl(slot, leader);
    if (follower) {
      slot = ls;
      found = ls >= 0;
    }
  }
  const uint64_t below = (1ull << lane) - 1ull;
  const uint64_t cm = __ballot(claimed);
  unsigned long long pbase = 0;
  if (lane == 0 && cm) pbase = atomicAdd(c.ctl + kCtlFreeHead, (unsigned long long)__popcll(cm));
  pbase = __shfl(pbase, 0);
  int u = -1;
  if (claimed) {
    const unsigned long long q = pbase + (unsigned long long)__popcll(cm & below);
    const unsigned long long fc = __hip_atomic_load(c.ctl + kCtlFreeCount, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (q < fc) u = (int)c.free_slots[q];
  }
  const uint64_t pm = __ballot(claimed && u >= 0);
  // (a tail lane past n is no failure either: it must not flag the cache full)
  const uint64_t fm = __ballot(found), xm = __ballot(slot < 0 && !deferred && active), sgm = __ballot(sighted);
  unsigned long long nbase = 0;
  if (st) {
    st->found += (uint32_t)__popcll(fm);
    st->claimed += (uint32_t)__popcll(cm);
    st->failed += (uint32_t)__popcll(xm);
    st->sighted += (uint32_t)__popcll(sgm);
  }
  if (lane == 0) {
    if (pm) nbase = atomicAdd(c.ctl + c.count_word, (unsigned long long)__popcll(pm));
    if (!st) {
      if (cm) atomicAdd(c.ctl + kCtlClaimed, (unsigned long long)__popcll(cm));
      if (fm) atomicAdd(c.ctl + kCtlFound, (unsigned long long)__popcll(fm));
      if (xm) atomicAdd(c.ctl + kCtlFailed, (unsigned long long)__popcll(xm));
      if (sgm) atomicAdd(c.ctl + kCtlSighted, (unsigned long long)__popcll(sgm));
    }
    // (a plain load first: a full cache under churn would otherwise have every wave exchange the same word)
    if ((cm != pm || xm) && __hip_atomic_load(c.ctl + kCtlFull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0)
      atomicExch(c.ctl + kCtlFull, 1ull);
  }
  nbase = __shfl(nbase, 0);
  if (claimed) {
    int4* e = c.entries + (size_t)slot * kCacheEntryGranules;
    e[0] = make_int4((int)a[0], (int)a[1], (int)a[2], (int)a[3]);
    e[1] = make_int4((int)a[4], (int)a[5], (int)a[6], (int)a[7]);
    e[2] = make_int4(0, 0, u, (int)c.epoch);  // valid once cache_flip_kernel has run (after the payload's build)
    if (u >= 0) c.new_list[nbase + (unsigned long long)__popcll(pm & below)] = make_uint4((uint32_t)slot, (uint32_t)u, 0u, 0u);
  }
  return slot;
}

// The record's entry is usable: valid and the key bytes equal. ok = A's decode verdict, u = payload index. A hit records
// this launch's epoch in the entry (the compaction keeps the most recently used entries).
__device__ AT2V_INLINE bool cache_hit(const CacheArgs& c, int slot, const uint32_t Aw[8], int& ok, int& u) {
  ok = 0;
  u = 0;
  if (slot < 0) return false;
  int4* e = c.entries + (size_t)slot * kCacheEntryGranules;
  const int4 k0 = e[0], k1 = e[1], m = e[2];
  ok = m.x;
  u = m.z;
  const bool hit = m.y == 1 && m.z >= 0 && (uint32_t)k0.x == Aw[0] && (uint32_t)k0.y == Aw[1] &&
                   (uint32_t)k0.z == Aw[2] && (uint32_t)k0.w == Aw[3] && (uint32_t)k1.x == Aw[4] &&
                   (uint32_t)k1.y == Aw[5] && (uint32_t)k1.z == Aw[6] && (uint32_t)k1.w == Aw[7];
  if (hit && (uint32_t)m.w != c.epoch) reinterpret_cast<int*>(e + 2)[3] = (int)c.epoch;
  if (!hit) u = 0;
  return hit;
}

// Verdict bits of a partitioned launch's wave (kPart: records in list order). When the wave's 64 records are 64
// consecutive records starting at a multiple of 64 (a list segment appended by one classify wave whose records all went
// to that list: the common case), lane 0 ORs two whole words; otherwise every valid record ORs its own bit. (64 atomics
// on the same two words from one instruction serialise in L2: +20% on a 1M-record comb launch, profiles/r05e.)
__device__ AT2V_INLINE void verdict_or(uint32_t* __restrict__ verdicts, uint32_t rec, int good, bool act, int lane) {
  const uint32_t r0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)rec);
  const int contig = __builtin_amdgcn_readfirstlane(__all(act && rec == r0 + (uint32_t)lane) && (r0 & 63u) == 0 ? 1 : 0);
  if (contig) {
    const uint64_t m = __ballot(good);
    if (lane == 0) {
      if ((uint32_t)m)
        __hip_atomic_fetch_or(verdicts + (r0 >> 5), (uint32_t)m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((uint32_t)(m >> 32))
        __hip_atomic_fetch_or(verdicts + (r0 >> 5) + 1, (uint32_t)(m >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  } else if (good && act) {
    __hip_atomic_fetch_or(verdicts + (rec >> 5), 1u << (rec & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Half-size verification: one chunk of 64 records per wave, no final inversion. kCache: the per-sender A
// cache is on; a wave whose 64 records all hit it skips decoding A and building [j]A (slot_of / cache from
// cache_lookup_kernel + cache_build_kernel, launched just before on the same stream).
// The body is a device function under two kernels with their own parameter lists, so the uncached kernel keeps exactly
// round 2's signature and code (an extra-parameter template of it measured ~1% slower: profiles/r03b, r03d).
// kComb (with kCache): entries carry per-key combs (at2v_comb.h); a wave whose 64 records all hit verifies from them
// (additions only), any other wave runs the uncached half-size path.
// kPart (partitioned cached launches, at2v_cache.h PartArgs): chunks are 64 entries of the classify kernel's lists
// instead of 64 consecutive records: with kCache ([j]A tables) the hit list's chunks (every record cached: A's decode and
// table skipped) and then the miss list's, without it the miss list alone (the comb kernel takes the hits). A record's
// verdict bit is set by an atomic OR (the lists are in no particular order; the launcher zeroed the words).
// kStaged (StagedArgs, the host pipeline's single launch): record i of region u = i >> ushift is read from the region's
// own layout once the host has published the region (stage_wait); a wave that cannot get it (abort, time limit) stores
// zero verdict words for its chunks.
constexpr unsigned long long kStageTimeoutTicks = 1000000000ull;  // 10 s of the 100 MHz s_memrealtime clock

// lane 0 polls the published region count until it exceeds `need` - 1; returns it (wave-uniform), or 0 on abort / time
// limit (then *dead)
__device__ AT2V_INLINE uint32_t stage_wait(const StagedArgs* sp, uint32_t need, int lane, bool& dead) {
  int got = 0;
  if (lane == 0) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
      const unsigned long long v = __hip_atomic_load(sp->ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      const uint32_t cnt = (uint32_t)v;
      if ((uint32_t)(v >> 32) == sp->epoch) {
        if (cnt & 0x80000000u) {
          got = -1;
          break;
        }
        if (cnt >= need) {
          got = (int)cnt;
          break;
        }
      }
      if (__builtin_amdgcn_s_memrealtime() - t0 > kStageTimeoutTicks) {
        __hip_atomic_store(sp->timeout, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        got = -1;
        break;
      }
      for (uint32_t z = 0; z < sp->nap; ++z) __builtin_amdgcn_s_sleep(8);
    }
  }
  got = __builtin_amdgcn_readfirstlane(got);
#ifndef AT2V_STAGE_FENCE
#define AT2V_STAGE_FENCE 2  // after every poll: 1 a system-scope acquire, 2 a workgroup-scope one (L1), 0 none
#endif
#if AT2V_STAGE_FENCE == 1
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope
#elif AT2V_STAGE_FENCE == 2
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
#endif
  dead = got < 0;
  return got < 0 ? 0u : (uint32_t)got;
}

template <bool kCache, bool kComb = false, bool kPart = false, bool kStaged = false>
__device__ AT2V_INLINE void verify_chunks(
    int4* astage, int4* rstage, const uint8_t* __restrict__ pk, const uint8_t* __restrict__ sig,
    const uint8_t* __restrict__ msg, uint32_t msg_total, const uint32_t* __restrict__ off, uint32_t n, int policy,
    uint32_t* __restrict__ verdicts, int4* __restrict__ scratch, const int4* __restrict__ btab,
    const int4* __restrict__ btab24, uint32_t* __restrict__ chunk_queue, const CacheArgs* cp,
    const PartArgs* pp = nullptr, const StagedArgs* sp = nullptr) {
  const int lane = threadIdx.x & 63;
  const int wib = AT2V_UNIFORM(threadIdx.x >> 6);  // wave-uniform: the LDS stage addresses live in SGPRs
  const uint32_t wave = blockIdx.x * kWavesPerBlock + wib;
  const uint32_t nwaves = gridDim.x * kWavesPerBlock;
  uint32_t nchunks = (n + 63) / 64;
  const uint32_t nwords = (n + 31) / 32;
  uint32_t nh = 0, nm = 0, hchunks = 0;
  if constexpr (kPart) {  // the list sizes the classify kernel left (same stream: complete)
    nh = kCache ? __builtin_amdgcn_readfirstlane(pp->counts[0]) : 0u;
    nm = __builtin_amdgcn_readfirstlane(pp->counts[1]);
    hchunks = (nh + 63) / 64;
    nchunks = hchunks + (nm + 63) / 64;
  }
#ifndef AT2V_MSG_TOUCH
#define AT2V_MSG_TOUCH 0  // 1: early loads of each lane's message sectors (consumed at SHA-512), see verify_chunks
#endif
#ifndef AT2V_EXP_SLOT_WAVES
#define AT2V_EXP_SLOT_WAVES 0  // EXPERIMENT ONLY (wrong verdicts): > 0 = waves share AT2V_EXP_SLOT_WAVES table slots, so the
                               // tables' footprint is L2-resident; measures what the table traffic costs in time/clock
#endif
#if AT2V_EXP_SLOT_WAVES
  int4* slot = scratch + ((size_t)(wave % AT2V_EXP_SLOT_WAVES) * 64 + lane) * kLaneGranules;
#else
  int4* slot = scratch + ((size_t)wave * 64 + lane) * kLaneGranules;
#endif
  const int4* ident = btab + (size_t)kNumBtabs * kBtabEntries * 8;  // shared identity entry after the B tables
  DevTabA ta{slot, astage + wib * 640, lane, ident};
  DevTabA tr{slot + kTabAGranules, rstage + wib * 640, lane, ident};
#if AT2V_LADDER_BW == 24  // the shared 24-bit tables [j]B and [j 2^144]B (kLadderEntries each, at2v_api.hip)
  const DevTabB tb0{btab24, astage + wib * 640, lane};                        // staged where A's entry was
  const DevTabB tb1{btab24 + (size_t)kLadderEntries * 8, rstage + wib * 640, lane};  // in R's stage
#else
  (void)btab24;
  const DevTabB tb0{btab, astage + wib * 640, lane};                      // [j]B, staged where A's entry was
  const DevTabB tb1{btab + (size_t)kBtabEntries * 8, rstage + wib * 640, lane};  // [j 2^128]B, in R's stage
#endif
  auto wmax = [](int v) { return wave_max_i32(v); };
#if AT2V_FAIR
  uint32_t* prog_lines = chunk_queue + 16;
  Pace pace{prog_lines + (size_t)wave * 16, prog_lines + (size_t)(wave ^ 4) * 16, 0u, 0u,
            (wib >= 4 && AT2V_FAIR_LAG > 0) ? AT2V_FAIR_LAG : 0};
  if (lane == 0) __hip_atomic_store(pace.mine, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
  NoPace pace;
#endif
  // Chunk c = wave first, then chunks nwaves + ticket from the per-launch queue counter (zeroed by the
  // launcher). The two waves of a SIMD do not get equal issue shares (arbitration by priority, then age), so
  // with a static c += nwaves split half the waves finished at 60% of the kernel time and their SIMDs ran the
  // rest on one wave at half throughput (tools/phase_bench wave timeline). Pulling chunks keeps
  // both waves busy until the queue drains. The ticket is a vector atomic from lane 0, broadcast with
  // readfirstlane, so the loop stays wavefront-uniform; every wave leaves after one ticket >= the chunk count.
  // First chunks: waves 0..3 of every block (one per SIMD) come before waves 4..7, so a launch with at most
  // 4 chunks per block runs every chunk on a SIMD of its own (blocks take the whole LDS: one per CU).
  constexpr uint32_t kHalf = kWavesPerBlock / 2;
  const uint32_t c_first = wib < (int)kHalf ? blockIdx.x * kHalf + wib
                                            : gridDim.x * kHalf + blockIdx.x * kHalf + (wib - kHalf);
  const uint8_t* const arena = pk;  // kStaged: the launch passes its arena as pk
  uint32_t known = 0;  // kStaged: regions this wave has seen published
  bool dead = false;   // kStaged: the regions it waits for will not come
  for (uint32_t c = c_first; c < nchunks;) {
    AT2V_PHASE(0);
#ifdef AT2V_WAIT_PROBE
    const unsigned long long t_chunk0 = __builtin_amdgcn_s_memtime();
#endif
    uint32_t i, ii;
    bool act;
    int phit = 0;        // kPart: a hit-list chunk (wave-uniform)
    uint32_t pinfo = 0;  // kPart: the hit's (payload << 1) | A's decode verdict
    if constexpr (kPart) {
      phit = c < hchunks ? 1 : 0;
      const uint32_t pos = (phit ? c : c - hchunks) * 64 + lane, cnt = phit ? nh : nm;
      const uint32_t pc = pos < cnt ? pos : cnt - 1;  // tail lanes recompute the list's last record; masked
      act = pos < cnt;
      i = ii = (phit ? pp->hidx : pp->midx)[pc];
      if (phit) pinfo = pp->hinfo[pc];
    } else {
      i = c * 64 + lane;
      ii = i < n ? i : n - 1;  // tail lanes recompute a real record; their bit is masked
      act = i < n;
    }
    int skip = 0;  // kStaged: the chunk's region never came (verdicts 0)
    if constexpr (kStaged) {  // the chunk's region (wave-uniform: regions are multiples of 64 records)
      const uint32_t u0 = (c * 64) >> sp->ushift, u = u0 < sp->nreg - 1 ? u0 : sp->nreg - 1;
      if (u >= known && !dead) known = stage_wait(sp, u + 1, lane, dead);
      skip = u >= known ? 1 : 0;
      const uint8_t* b = arena + sp->at[u];
      const uint32_t rc = u == sp->nreg - 1 ? sp->last_c : 1u << sp->ushift;
      pk = b;
      sig = b + (size_t)rc * 32;
      off = reinterpret_cast<const uint32_t*>(b + (size_t)rc * 96);
      msg = b + (((size_t)rc * 96 + ((size_t)rc + 1) * 4 + 15) & ~(size_t)15);
      msg_total = sp->mb[u];
      ii -= u << sp->ushift;
    }
    uint32_t Rw[8], Sw[8], Aw[8];
    load8(Rw, sig + (size_t)ii * 64);
    load8(Sw, sig + (size_t)ii * 64 + 32);
    load8(Aw, pk + (size_t)ii * 32);
    const uint32_t o0 = off[ii];
    const uint32_t len = off[ii + 1] - o0;
#ifdef AT2V_WAIT_PROBE
    AT2V_PROBE(pace.probe[2], asm volatile("s_waitcnt vmcnt(0)" ::: "memory"));
#endif
    // message words: a wave whose messages all end >= 8 bytes before the buffer end reads two aligned words and
    // funnel-shifts them (no per-lane branch); otherwise every byte is bounds-checked (the last records of a batch)
    const int msg_fast =
        __builtin_amdgcn_readfirstlane(__all((uint64_t)o0 + len + 8 <= (uint64_t)msg_total) ? 1 : 0);
    const uint32_t* mw = reinterpret_cast<const uint32_t*>(msg) + (o0 >> 2);
    const uint32_t msh = (o0 & 3u) * 8;
    auto msg_unguarded = [=](uint32_t j) -> uint32_t { return __builtin_amdgcn_alignbit(mw[j + 1], mw[j], msh); };
    auto msg_guarded = [=](uint32_t j) -> uint32_t {
      const uint32_t a = o0 + 4 * j;
      const uint32_t a0 = a & ~3u, sh = (a & 3u) * 8;
      const uint32_t lo = load_u32_guarded(msg, a0, msg_total);
      if (sh == 0) return lo;
      const uint32_t hi = load_u32_guarded(msg, a0 + 4, msg_total);
      return __builtin_amdgcn_alignbit(hi, lo, sh);
    };
#if AT2V_MSG_TOUCH
    // Touch the first three 64-byte sectors of the lane's message now, so SHA-512 (after the two decodes) finds them in
    // cache: its message loads are issued one at a time, each behind its own wait. The words are consumed by an empty asm
    // statement at the start of SHA-512 (so the loads are kept and their wait lands there, long after they returned).
    uint32_t touch[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const uint32_t a = o0 + (64u * q < len ? 64u * q : (len ? len - 1 : 0u));
      touch[q] = msg_total ? *reinterpret_cast<const uint32_t*>(msg + ((a < msg_total ? a : msg_total - 1) & ~3u)) : 0u;
    }
    auto touched = [=]() { asm volatile("" ::"v"(touch[0]), "v"(touch[1]), "v"(touch[2])); };
#else
    auto touched = [] {};
#endif
    MsgSplit<decltype(msg_unguarded), decltype(msg_guarded), decltype(touched)> msgword{msg_fast, msg_unguarded,
                                                                                        msg_guarded, touched};
#if AT2V_FIELD_FU
    int good;
    if (kCache) {
      const CacheArgs& cc = *cp;
      int a_ok = 0, u = 0, all_hit;
      if constexpr (kPart) {  // classified already
        all_hit = phit;
        a_ok = (int)(pinfo & 1u);
        u = (int)(pinfo >> 1);
      } else {
        // the chunk's senders: looked up (new keys claimed for the build stream) in the chunk prologue
        const int slot = cache_lookup_wave(cc, Aw, lane, i < n);
        const bool hit = cache_hit(cc, slot, Aw, a_ok, u);
        all_hit = __builtin_amdgcn_readfirstlane(__all(hit) ? 1 : 0);
        if (lane == 0) {
          atomicAdd(cc.ctl + kCtlChunks, 1ull);
          if (all_hit) atomicAdd(cc.ctl + kCtlChunkHits, 1ull);
        }
      }
      if (kComb) {
        if (all_hit) {
          const DevComb tc{cc.payload + (size_t)u * (kCombBytes / 16), {astage + wib * 640, rstage + wib * 640}, lane};
          const DevBCombLat tbc{cc.bcomb_lat, {astage + wib * 640, rstage + wib * 640}, lane};
          good = verify_comb_fu(Rw, Aw, Sw, len, msgword, policy, a_ok, tc, tbc) & act;
        } else {
          good = verify_half_fu<false, AT2V_LADDER_BW>(Rw, Aw, Sw, len, msgword, policy, ta, tr, tb0, tb1, wmax, pace) &
                 act;
        }
      } else {
        DevTabA tc{ta};
        if (all_hit) tc.base = cc.payload + (size_t)u * kTabAGranules;
        good = verify_half_fu<true, AT2V_LADDER_BW>(Rw, Aw, Sw, len, msgword, policy, tc, tr, tb0, tb1, wmax, pace,
                                                     all_hit, a_ok) &
               act;
      }
    } else if (skip) {
      good = 0;
    } else {
      good = verify_half_fu<false, AT2V_LADDER_BW>(Rw, Aw, Sw, len, msgword, policy, ta, tr, tb0, tb1, wmax, pace) & act;
    }
#else
    const int good = verify_half(Rw, Aw, Sw, len, msgword, policy, ta, tr, tb0, tb1, wmax, pace) & (i < n);
#endif
    const uint64_t mask = __ballot(good);
#ifdef AT2V_WAIT_PROBE
    AT2V_WAIT_PROBE_SINK(ta.waited + tr.waited, tb0.waited + tb1.waited, pace.probe[0], pace.probe[1],
                         __builtin_amdgcn_s_memtime() - t_chunk0, ta.lds_waited + tr.lds_waited, pace.probe[2]);
    ta.waited = tr.waited = tb0.waited = tb1.waited = ta.lds_waited = tr.lds_waited = tb0.lds_waited = tb1.lds_waited = 0;
    pace.probe[0] = pace.probe[1] = pace.probe[2] = 0;
#endif
    uint32_t ticket = 0;
    if constexpr (kPart) {  // records in list order
      verdict_or(verdicts, i, good, act, lane);
    } else if (lane == 0) {
      verdicts[2 * c] = (uint32_t)mask;
      if (2 * c + 1 < nwords) verdicts[2 * c + 1] = (uint32_t)(mask >> 32);
    }
    if (lane == 0) {
#if AT2V_QUEUE
#if AT2V_SOLO_TAIL
      // the last nwaves/2 chunks go to waves 0..3 only: their SIMD partners leave, so each of those chunks
      // runs on one wave per SIMD instead of ending as a partnerless straggler
      if (wib >= (int)kHalf &&
          __hip_atomic_load(chunk_queue, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + nwaves + nwaves / 2 >= nchunks)
        ticket = nchunks;
      else
#endif
        ticket = atomicAdd(chunk_queue, 1u);
#endif
    }
#if AT2V_QUEUE
    ticket = __builtin_amdgcn_readfirstlane(ticket);
    c = ticket < nchunks ? nwaves + ticket : nchunks;  // no wrap: ticket < nchunks <= 2^26
#else
    c += nwaves;
#endif
    AT2V_PHASE(6);
  }
}

__global__ __launch_bounds__(kBlock, AT2V_VERIFY_WAVES_PER_SIMD) void verify_kernel(
    const uint8_t* __restrict__ pk, const uint8_t* __restrict__ sig, const uint8_t* __restrict__ msg,
    uint32_t msg_total, const uint32_t* __restrict__ off, uint32_t n, int policy, uint32_t* __restrict__ verdicts,
    int4* __restrict__ scratch, const int4* __restrict__ btab, const int4* __restrict__ btab24,
    uint32_t* __restrict__ chunk_queue) {
  __shared__ int4 astage[kWavesPerBlock * 10 * 64];
  __shared__ int4 rstage[kWavesPerBlock * 10 * 64];
  verify_chunks<false>(astage, rstage, pk, sig, msg, msg_total, off, n, policy, verdicts, scratch, btab, btab24,
                       chunk_queue, nullptr);
}

// the same with the per-sender A cache (at2v_opts.sender_cache, tables [j]A)
// the host pipeline's single launch over a batch still being uploaded (StagedArgs)
__global__ __launch_bounds__(kBlock, AT2V_VERIFY_WAVES_PER_SIMD) void verify_kernel_staged(
    const uint8_t* __restrict__ arena, uint32_t n, int policy, uint32_t* __restrict__ verdicts,
    int4* __restrict__ scratch, const int4* __restrict__ btab, const int4* __restrict__ btab24,
    uint32_t* __restrict__ chunk_queue, StagedArgs sa) {
  __shared__ int4 astage[kWavesPerBlock * 10 * 64];
  __shared__ int4 rstage[kWavesPerBlock * 10 * 64];
  // one system-scope acquire per block before any wave reads a region: no cache keeps a line of the arena from an
  // earlier launch (the regions are re-uploaded at the same addresses every call)
  if (threadIdx.x < 64) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  __syncthreads();
  verify_chunks<false, false, false, true>(astage, rstage, arena, arena, arena, 0, nullptr, n, policy, verdicts,
                                           scratch, btab, btab24, chunk_queue, nullptr, nullptr, &sa);
}

__global__ __launch_bounds__(kBlock, AT2V_VERIFY_WAVES_PER_SIMD) void verify_kernel_cached(
    const uint8_t* __restrict__ pk, const uint8_t* __restrict__ sig, const uint8_t* __restrict__ msg,
    uint32_t msg_total, const uint32_t* __restrict__ off, uint32_t n, int policy, uint32_t* __restrict__ verdicts,
    int4* __restrict__ scratch, const int4* __restrict__ btab, const int4* __restrict__ btab24,
    uint32_t* __restrict__ chunk_queue, CacheArgs c) {
  __shared__ int4 astage[kWavesPerBlock * 10 * 64];
  __shared__ int4 rstage[kWavesPerBlock * 10 * 64];
  verify_chunks<true>(astage, rstage, pk, sig, msg, msg_total, off, n, policy, verdicts, scratch, btab, btab24,
                      chunk_queue, &c);
}

// Partitioned cached launches (at2v_cache.h PartArgs): the ladder over the classify kernel's miss list (sender_comb: the
// comb kernel below takes the hits) or over both lists ([j]A tables: hit chunks skip A's decode and table)
__global__ __launch_bounds__(kBlock, AT2V_VERIFY_WAVES_PER_SIMD) void verify_kernel_miss(
    const uint8_t* __restrict__ pk, const uint8_t* __restrict__ sig, const uint8_t* __restrict__ msg,
    uint32_t msg_total, const uint32_t* __restrict__ off, uint32_t n, int policy, uint32_t* __restrict__ verdicts,
    int4* __restrict__ scratch, const int4* __restrict__ btab, const int4* __restrict__ btab24,
    uint32_t* __restrict__ chunk_queue, PartArgs p) {
  __shared__ int4 astage[kWavesPerBlock * 10 * 64];
  __shared__ int4 rstage[kWavesPerBlock * 10 * 64];
  verify_chunks<false, false, true>(astage, rstage, pk, sig, msg, msg_total, off, n, policy, verdicts, scratch, btab,
                                    btab24, chunk_queue, nullptr, &p);
}
__global__ __launch_bounds__(kBlock, AT2V_VERIFY_WAVES_PER_SIMD) void verify_kernel_tables_part(
    const uint8_t* __restrict__ pk, const uint8_t* __restrict__ sig, const uint8_t* __restrict__ msg,
    uint32_t msg_total, const uint32_t* __restrict__ off, uint32_t n, int policy, uint32_t* __restrict__ verdicts,
    int4* __restrict__ scratch, const int4* __restrict__ btab, const int4* __restrict__ btab24,
    uint32_t* __restrict__ chunk_queue, CacheArgs c, PartArgs p) {
  __shared__ int4 astage[kWavesPerBlock * 10 * 64];
  __shared__ int4 rstage[kWavesPerBlock * 10 * 64];
  verify_chunks<true, false, true>(astage, rstage, pk, sig, msg, msg_total, off, n, policy, verdicts, scratch, btab,
                                   btab24, chunk_queue, &c, &p);
}

// The classify kernel of a partitioned cached launch: one record per lane, a wave takes kClassifyGroups consecutive
// 64-record groups (a block of 4 waves, 4 kClassifyGroups groups). Every sender is looked up exactly as the round-4
// kernels did in their chunk prologue (cache_lookup_wave: claims, sightings, epochs); the block then takes room in the
// two lists with one atomic per list and writes its hits (index, payload, decode verdict) and misses in group order,
// and adds its statistics with one atomic per counter. (One wave per group with per-wave atomics took 0.54-0.77 ms per
// 1M records: ~100k atomics on a handful of control words, profiles/r05f. Eight groups per wave and per-wave list
// atomics: the same atomic count as now, but each wave ran eight dependent lookup chains one after the other.)
// Block shape: AT2V_CLASSIFY_WAVES waves x AT2V_CLASSIFY_GROUPS groups. Blocks of 16 waves x 4 groups (8x fewer list and
// statistics atomics on the same control words) measured no better on the distinct-key leg (0.977 against 0.982-0.987
// of plain, profiles/r05zi): the atomics are not what the classify kernel waits for.
#ifndef AT2V_CLASSIFY_GROUPS
#define AT2V_CLASSIFY_GROUPS 2
#endif
#ifndef AT2V_CLASSIFY_WAVES
#define AT2V_CLASSIFY_WAVES 4
#endif
constexpr int kClassifyGroups = AT2V_CLASSIFY_GROUPS;
constexpr int kClassifyWaves = AT2V_CLASSIFY_WAVES;
__global__ __launch_bounds__(64 * AT2V_CLASSIFY_WAVES) void cache_classify_kernel(const uint8_t* __restrict__ pk,
                                                                                 uint32_t n, CacheArgs c, PartArgs p) {
  __shared__ uint32_t sstat[kClassifyWaves][8];
  __shared__ uint32_t sbase[2];
  const int lane = threadIdx.x & 63;
  const int wib = threadIdx.x >> 6;
  const uint32_t ngroups = (n + 63) / 64;
  const uint32_t g0 = (blockIdx.x * kClassifyWaves + (uint32_t)wib) * kClassifyGroups;
  LookupStats st;
  uint64_t hm[kClassifyGroups], am[kClassifyGroups];
  uint32_t info[kClassifyGroups];
  uint32_t nh = 0, na = 0, chunks = 0, chunk_hits = 0;
#pragma unroll
  for (int g = 0; g < kClassifyGroups; ++g) {
    hm[g] = am[g] = 0;
    info[g] = 0;
    if (g0 + g < ngroups) {  // wave-uniform
      const uint32_t i = (g0 + g) * 64 + lane;
      const bool active = i < n;
      uint32_t Aw[8];
      load8(Aw, pk + (size_t)(active ? i : n - 1) * 32);
      const int slot = cache_lookup_wave(c, Aw, lane, active, &st);
      int a_ok = 0, u = 0;
      const bool hit = cache_hit(c, slot, Aw, a_ok, u) && active;
      am[g] = __ballot(active);
      hm[g] = __ballot(hit);
      info[g] = ((uint32_t)u << 1) | (uint32_t)(a_ok & 1);
      nh += (uint32_t)__popcll(hm[g]);
      na += (uint32_t)__popcll(am[g]);
      ++chunks;
      chunk_hits += hm[g] == am[g] ? 1u : 0u;
    }
  }
  if (lane == 0) {
    sstat[wib][0] = chunks;
    sstat[wib][1] = chunk_hits;
    sstat[wib][2] = nh;
    sstat[wib][3] = st.found;
    sstat[wib][4] = st.claimed;
    sstat[wib][5] = st.failed;
    sstat[wib][6] = st.sighted;
    sstat[wib][7] = na - nh;
  }
  __syncthreads();
  if (threadIdx.x == 0) {  // the block's room in the two lists
    uint32_t th = 0, tm = 0;
    for (int w = 0; w < kClassifyWaves; ++w) {
      th += sstat[w][2];
      tm += sstat[w][7];
    }
    sbase[0] = th ? atomicAdd(p.counts, th) : 0u;
    sbase[1] = tm ? atomicAdd(p.counts + 1, tm) : 0u;
  }
  if (threadIdx.x < 7) {
    uint32_t v = 0;
    for (int w = 0; w < kClassifyWaves; ++w) v += sstat[w][threadIdx.x];
    const int k = threadIdx.x;
    const int word = k == 0 ? kCtlChunks : k == 1 ? kCtlChunkHits : k == 2 ? kCtlRecHits : k == 3 ? kCtlFound
                     : k == 4 ? kCtlClaimed : k == 5 ? kCtlFailed : kCtlSighted;
    if (v) atomicAdd(c.ctl + word, (unsigned long long)v);
  }
  __syncthreads();
  uint32_t hb = sbase[0], mb = sbase[1];
  for (int w = 0; w < wib; ++w) {  // (wave-uniform) the earlier waves' shares of the block's room
    hb += sstat[w][2];
    mb += sstat[w][7];
  }
  const uint64_t below = (1ull << lane) - 1ull;
#pragma unroll
  for (int g = 0; g < kClassifyGroups; ++g) {
    const uint32_t i = (g0 + g) * 64 + lane;
    const uint64_t mm = am[g] & ~hm[g];
    if ((hm[g] >> lane) & 1ull) {
      const uint32_t q = hb + (uint32_t)__popcll(hm[g] & below);
      p.hidx[q] = i;
      p.hinfo[q] = info[g];
    } else if ((mm >> lane) & 1ull) {
      p.midx[mb + (uint32_t)__popcll(mm & below)] = i;
    }
    hb += (uint32_t)__popcll(hm[g]);
    mb += (uint32_t)__popcll(mm);
  }
}

// LDS words of the four-wave split check (in the kernel's `part` array, word-major: [word][lane])
constexpr int kSplitDig = 0;          // c0 digits (8 words), |c1| digits (8 words)
constexpr int kSplitFlags = 16 * 64;  // bit 0: the lattice / window check, bit 1: c1 < 0
constexpr int kSplitP1 = 40 * 64;     // [c1]R, cached form (40 words)
constexpr int kSplitPb = 80 * 64;     // -[t]B, cached form (40 words)

// Low-latency verify from combs (at2v_opts.sender_comb, launches of <= small_batch_max records): a block of 4 waves (one
// per SIMD) owns a chunk of 64 records. Wave 0 looks the chunk's senders up (claiming new keys for the build stream) and
// hands each record's entry (payload index or -1, decode verdict) to the other waves through LDS, so all four waves take
// the same branch. A chunk whose records all hit splits each record's work by wave (at2v_comb.h, comb_check_split):
//   wave 0: decode R and check its canonicity (one exponentiation), then, after the barrier, R' = Pa0 + Pa1 + Pb and
//           the projective comparison -> verdict words
//   wave 1: s < l, the kBCombPos (11) B-comb additions -> Pb
//   wave 2: SHA-512 -> k, A-comb positions 0..15 -> Pa0;   wave 3: SHA-512 -> k, positions 16..31 -> Pa1
// so a record's latency is the longest part (SHA-512 + 13 additions) instead of SHA-512 + 37 additions + an inversion.
// Any other chunk (a sender seen for the first time: its comb is built on the build stream after this launch and serves
// later launches; a claim without a payload; a probe failure) runs the half-size check V = [c0]A + [c1]R - [t]B = 0
//  split over the four waves: wave 0 decodes A and builds [j]A, wave 1 decodes R and builds [j]R while
// wave 2 hashes (SHA-512 -> k), reduces the lattice (c0, c1, t) and hands the digits over LDS; then wave 0 runs the
// [c0]A ladder, wave 1 the [c1]R ladder (four doublings and one addition per window), wave 2 adds [t]B from the comb of
// B, and wave 0 checks the sum. The chain of a record is then decode + table + one 128-bit ladder, instead of SHA-512,
// the lattice and the fixed-base additions on top (the two-lane split of the pair kernel). A first-seen
// sender costs this instead of waiting for its comb (round 3: 0.82-0.94 ms of device time, profiles/r03zg).
// Verdict words are written by wave 0's lane 0 for every chunk.
constexpr int kLatBlock = 256;
__global__ __launch_bounds__(kLatBlock, 1) void verify_comb_lat_kernel(
    const uint8_t* __restrict__ pk, const uint8_t* __restrict__ sig, const uint8_t* __restrict__ msg,
    uint32_t msg_total, const uint32_t* __restrict__ off, uint32_t n, int policy, uint32_t* __restrict__ verdicts,
    int4* __restrict__ scratch, const int4* __restrict__ btab, CacheArgs c) {
  __shared__ int4 stage[4 * 2 * 640];        // per wave two 10 KiB LDS-DMA stages
  __shared__ uint32_t part[3 * 40 * 64];      // Pb, Pa0, Pa1 (p3, 40 words) per lane, word-major; or the R side's P1
  __shared__ uint32_t sok[64];                // wave 1's s < l, or the R side's checks
  __shared__ int sent[2 * 64];                // wave 0's cache outcome per record: payload index (-1: miss), A verdict
  __shared__ int snw;                         // split check: the chunk's window count (wave 2)
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int4* st0 = stage + (size_t)w * 2 * 640;
  int4* st1 = st0 + 640;
  const uint32_t nchunks = (n + 63) / 64, nwords = (n + 31) / 32;
  auto wmax = [](int v) { return wave_max_i32(v); };
  for (uint32_t c0 = blockIdx.x; c0 < nchunks; c0 += gridDim.x) {
    const uint32_t i = c0 * 64 + lane;
    const uint32_t ii = i < n ? i : n - 1;
    uint32_t Rw[8], Sw[8], Aw[8];
    load8(Rw, sig + (size_t)ii * 64);
    load8(Sw, sig + (size_t)ii * 64 + 32);
    load8(Aw, pk + (size_t)ii * 32);
    if (w == 0) {
      const int slot = cache_lookup_wave(c, Aw, lane, i < n);
      int a_ok0 = 0, u0 = 0;
      const bool hit0 = cache_hit(c, slot, Aw, a_ok0, u0);
      sent[lane] = hit0 ? u0 : -1;
      sent[64 + lane] = a_ok0;
    }
    __syncthreads();
    const int u = sent[lane], a_ok = sent[64 + lane];
    const int all_hit = __builtin_amdgcn_readfirstlane(__all(u >= 0) ? 1 : 0);  // the same in every wave (LDS)
    if (w == 0 && lane == 0) {
      atomicAdd(c.ctl + kCtlChunks, 1ull);
      if (all_hit) atomicAdd(c.ctl + kCtlChunkHits, 1ull);
    }
    const uint32_t o0 = off[ii];
    const uint32_t len = off[ii + 1] - o0;
    const int msg_fast =
        __builtin_amdgcn_readfirstlane(__all((uint64_t)o0 + len + 8 <= (uint64_t)msg_total) ? 1 : 0);
    const uint32_t* mw = reinterpret_cast<const uint32_t*>(msg) + (o0 >> 2);
    const uint32_t msh = (o0 & 3u) * 8;
    auto msg_unguarded = [=](uint32_t j) -> uint32_t { return __builtin_amdgcn_alignbit(mw[j + 1], mw[j], msh); };
    auto msg_guarded = [=](uint32_t j) -> uint32_t {
      const uint32_t a = o0 + 4 * j;
      const uint32_t a0 = a & ~3u, sh = (a & 3u) * 8;
      const uint32_t lo = load_u32_guarded(msg, a0, msg_total);
      if (sh == 0) return lo;
      const uint32_t hi = load_u32_guarded(msg, a0 + 4, msg_total);
      return __builtin_amdgcn_alignbit(hi, lo, sh);
    };
    auto touched = [] {};
    MsgSplit<decltype(msg_unguarded), decltype(msg_guarded), decltype(touched)> msgword{msg_fast, msg_unguarded,
                                                                                        msg_guarded, touched};
    gu_p3 R;   // all-hit: wave 0's decoded R;  fallback: wave 0's decoded A, then [c0]A
    int ok0 = 0;
    uint32_t td[kBCombLatDigitWords];  // fallback, wave 2: t's digits for the (low-latency) comb of B
    int4* slot = scratch + (((size_t)blockIdx.x * kWavesPerBlock + w) * 64 + lane) * kLaneGranules;
    const DevTabA tp{slot, st0, lane, btab + (size_t)kNumBtabs * kBtabEntries * 8};
    if (all_hit) {
      if (w == 0) {
        ok0 = comb_decode_r(R, Rw) & comb_prechecks(Rw, Aw, Sw, policy, a_ok);
      } else {
        gu_p3 P;
        gu_p3_identity(P);
        if (w == 1) {
          sok[lane] = (uint32_t)sc_is_canonical(Sw);
          uint32_t sd[kBCombLatDigitWords];
          bcomb_recode<kBCombLatBits>(sd, Sw);
          const DevBCombLat tb{c.bcomb_lat, {st0, st1}, lane};
          comb_sum<false>(P, sd, 0, kBCombLatPos, tb);
        } else {
          uint32_t kd[kCombDigitWords];
          comb_k_digits(kd, Rw, Aw, len, msgword);
          const DevComb tc{c.payload + (size_t)u * (kCombBytes / 16), {st0, st1}, lane};
          comb_sum<true>(P, kd, w == 2 ? 0 : kCombPos / 2, w == 2 ? kCombPos / 2 : kCombPos, tc);
        }
        const uint32_t* pw = reinterpret_cast<const uint32_t*>(&P);
        uint32_t* dst = part + (size_t)(w - 1) * 40 * 64;
#pragma unroll
        for (int q = 0; q < 40; ++q) dst[q * 64 + lane] = pw[q];
      }
    } else if (w == 0) {  // split check, phase 1: V1, the policy pre-checks, A decoded (dalek rules) and [j]A
      ok0 = split_a_side(R, Rw, Aw, Sw, policy, tp);
    } else if (w == 1) {  // R canonical and decoded, [j]R (c1's sign is applied per digit in phase 2)
      sok[lane] = (uint32_t)split_r_side(Rw, tp);
    } else if (w == 2) {  // k = SHA-512(R || A || M) mod l, the lattice (c0, c1), t = c1 s mod l: digits to LDS
      uint32_t c0d[8], c1d[8];
      int c1_neg, nw_lane;
      const int okl = split_scalars(c0d, c1d, td, c1_neg, nw_lane, Rw, Aw, Sw, len, msgword);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        part[kSplitDig + q * 64 + lane] = c0d[q];
        part[kSplitDig + (8 + q) * 64 + lane] = c1d[q];
      }
      part[kSplitFlags + lane] = (uint32_t)okl | ((uint32_t)c1_neg << 1);
      const int nw = wmax(nw_lane);
      if (lane == 0) snw = nw < 1 ? 1 : nw;
    }
    __syncthreads();
    if (!all_hit) {  // split check, phase 2: the two ladders and [t]B
      if (w < 2) {
        uint32_t cd[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) cd[q] = part[kSplitDig + (8 * w + q) * 64 + lane];
        const int flip = w == 1 ? (int)(part[kSplitFlags + lane] >> 1) & 1 : 0;
        gu_p3 P;
        split_side_ladder(P, cd, snw, flip, tp);
        if (w == 0) {
          R = P;
        } else {
          gu_cached cm;
          gu_p3_to_cached(cm, P);
          const uint32_t* cw = reinterpret_cast<const uint32_t*>(&cm);
#pragma unroll
          for (int q = 0; q < 40; ++q) part[kSplitP1 + q * 64 + lane] = cw[q];
        }
      } else if (w == 2) {
        gu_cached cm;
        split_neg_tb(cm, td, DevBCombLat{c.bcomb_lat, {st0, st1}, lane});  // -[t]B
        const uint32_t* cw = reinterpret_cast<const uint32_t*>(&cm);
#pragma unroll
        for (int q = 0; q < 40; ++q) part[kSplitPb + q * 64 + lane] = cw[q];
      }
    }
    __syncthreads();
    if (w == 0) {
      int good;
      if (all_hit) {
        gu_p3 Pb, Pa0, Pa1;
        uint32_t* pb = reinterpret_cast<uint32_t*>(&Pb);
        uint32_t* p0 = reinterpret_cast<uint32_t*>(&Pa0);
        uint32_t* p1 = reinterpret_cast<uint32_t*>(&Pa1);
#pragma unroll
        for (int q = 0; q < 40; ++q) {
          pb[q] = part[q * 64 + lane];
          p0[q] = part[40 * 64 + q * 64 + lane];
          p1[q] = part[80 * 64 + q * 64 + lane];
        }
        good = ok0 & (int)sok[lane] & comb_check_split(R, Pa0, Pa1, Pb) & (i < n);
      } else {  // V = [c0]A + [c1]R - [t]B == identity
        gu_cached c1r, cnb;
        uint32_t* w1 = reinterpret_cast<uint32_t*>(&c1r);
        uint32_t* w2 = reinterpret_cast<uint32_t*>(&cnb);
#pragma unroll
        for (int q = 0; q < 40; ++q) {
          w1[q] = part[kSplitP1 + q * 64 + lane];
          w2[q] = part[kSplitPb + q * 64 + lane];
        }
        good = ok0 & (int)sok[lane] & (int)(part[kSplitFlags + lane] & 1) & split_combine(R, c1r, cnb) & (i < n);
      }
      const uint64_t mask = __ballot(good);
      if (lane == 0) {
        verdicts[2 * c0] = (uint32_t)mask;
        if (2 * c0 + 1 < nwords) verdicts[2 * c0 + 1] = (uint32_t)(mask >> 32);
      }
    }
    __syncthreads();  // the LDS parts are reused by the block's next chunk
  }
}

// The message reader of one record (verify_chunks' MsgSplit: the fast form when the wave's messages all end 8 bytes
// before the buffer end), handed to body(msgword). A plain function, so the comb path below inlines it (as lambdas the
// compiler outlined these bodies into calls).
template <class Body>
__device__ AT2V_INLINE int with_msg_reader(const uint8_t* __restrict__ msg, uint32_t msg_total, uint32_t b0, uint32_t bl,
                                           Body&& body) {
#if AT2V_EXP_CONST_MSG  // EXPERIMENT (wrong verdicts, timing only): message words from registers, no message loads
  auto msg_const = [=](uint32_t j) -> uint32_t { return j * 0x01010101u + b0; };
  auto touched0 = [] {};
  MsgSplit<decltype(msg_const), decltype(msg_const), decltype(touched0)> mc{1, msg_const, msg_const, touched0};
  return body(mc);
#endif
  const int msg_fast = __builtin_amdgcn_readfirstlane(__all((uint64_t)b0 + bl + 8 <= (uint64_t)msg_total) ? 1 : 0);
  const uint32_t* mw = reinterpret_cast<const uint32_t*>(msg) + (b0 >> 2);
  const uint32_t msh = (b0 & 3u) * 8;
  auto msg_unguarded = [=](uint32_t j) -> uint32_t { return __builtin_amdgcn_alignbit(mw[j + 1], mw[j], msh); };
  auto msg_guarded = [=](uint32_t j) -> uint32_t {
    const uint32_t a = b0 + 4 * j;
    const uint32_t a0 = a & ~3u, sh = (a & 3u) * 8;
    const uint32_t lo = load_u32_guarded(msg, a0, msg_total);
    if (sh == 0) return lo;
    const uint32_t hi = load_u32_guarded(msg, a0 + 4, msg_total);
    return __builtin_amdgcn_alignbit(hi, lo, sh);
  };
  auto touched = [] {};
  MsgSplit<decltype(msg_unguarded), decltype(msg_guarded), decltype(touched)> msgword{msg_fast, msg_unguarded,
                                                                                      msg_guarded, touched};
  return body(msgword);
}

// R' of record i (clamped to the batch) from its key's comb; returns the checks that need no point arithmetic
template <class TabBC>
__device__ AT2V_INLINE int comb2_point(gu_p3& P, uint32_t i, uint32_t n, const uint8_t* __restrict__ pk,
                                       const uint8_t* __restrict__ sig, const uint8_t* __restrict__ msg,
                                       uint32_t msg_total, const uint32_t* __restrict__ off, int policy, int a_ok,
                                       const int4* __restrict__ comb_key, const TabBC& tbc, int4* sa, int4* sr,
                                       int lane
#ifdef AT2V_COMB_PROBE
                                       , CombProbe* pr = nullptr
#endif
) {
  const uint32_t ii = i < n ? i : n - 1;
  uint32_t Rw[8], Sw[8], Aw[8];
  int ok;
  uint32_t o0, len;
#ifdef AT2V_COMB_PROBE
  unsigned long long dummy = 0;
  unsigned long long& p_rec = pr ? pr->v[kCpRecord] : dummy;
  (void)p_rec;
#endif
  AT2V_CPROBE(p_rec, {
    load8(Rw, sig + (size_t)ii * 64);
    load8(Sw, sig + (size_t)ii * 64 + 32);
    load8(Aw, pk + (size_t)ii * 32);
    o0 = off[ii];
    len = off[ii + 1] - o0;
    ok = comb_prechecks(Rw, Aw, Sw, policy, a_ok);
  });
  const DevComb tc{comb_key, {sa, sr}, lane};
  with_msg_reader(msg, msg_total, o0, len, [&](auto& mwd) {
#ifdef AT2V_COMB_PROBE
    if (pr) {  // comb_point with its two phases timed apart
      uint32_t kd[kCombDigitWords], sd[BCombGeom<TabBC::kBits>::kDigitWords];
      AT2V_CPROBE(pr->v[kCpSha], {
        comb_k_digits(kd, Rw, Aw, len, mwd);
        bcomb_recode<TabBC::kBits>(sd, Sw);
      });
      AT2V_CPROBE(pr->v[kCpSums], {
        gu_p3_identity(P);
        comb_sum<true>(P, kd, 0, kCombPos, tc);
        comb_sum<false>(P, sd, 0, BCombGeom<TabBC::kBits>::kPos, tbc);
      });
      return 0;
    }
#endif
    comb_point(P, Rw, Aw, Sw, len, mwd, tc, tbc);
    return 0;
  });
#ifdef AT2V_COMB_PROBE
  if (pr) {
    pr->v[kCpAWait] += tc.waited;
    pr->v[kCpStage] += tc.stage_waited;
    pr->v[kCpLds] += tc.lds_waited;
  }
#endif
  return ok;
}

// comb2_point with the record's offset and length already known (the hit loop loads them with the list) and the message
// staged in LDS: its words go to the wave's second comb stage by LDS-DMA (one global_load_lds_dword per word, issued
// together with the loads of R, S and A), so the record pays one memory latency before SHA-512 instead of one for its
// loads and one per message block. Used when every lane's message (with one word of alignment slack) fits the stage's
// kMsgStageWords words and ends 8 bytes before the buffer end (the unguarded reader's condition); returns -1 without
// doing anything otherwise (the caller falls back to comb2_point).
constexpr int kMsgStageWords = 40;  // the 10 KiB stage: 40 words x 64 lanes x 4 B
template <class TabBC>
__device__ AT2V_INLINE int comb2_point_staged(gu_p3& P, uint32_t ii, uint32_t o0, uint32_t len,
                                              const uint8_t* __restrict__ pk, const uint8_t* __restrict__ sig,
                                              const uint8_t* __restrict__ msg, uint32_t msg_total, int policy, int a_ok,
                                              const int4* __restrict__ comb_key, const TabBC& tbc, int4* sa,
                                              int4* sr, int lane
#ifdef AT2V_COMB_PROBE
                                              , CombProbe* pr = nullptr
#endif
) {
  const uint32_t kl = (len >> 2) + 2;  // words 0 .. (len >> 2) + 1 of the aligned window (the reader reads j and j + 1)
  const int fits = __builtin_amdgcn_readfirstlane(
      __all((uint64_t)o0 + len + 8 <= (uint64_t)msg_total && kl <= (uint32_t)kMsgStageWords) ? 1 : 0);
  if (!fits) return -1;
  const int kw = wave_max_i32((int)kl);
  const uint32_t* mw = reinterpret_cast<const uint32_t*>(msg + (o0 & ~3u));
  uint32_t* const ml = reinterpret_cast<uint32_t*>(sr);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the stage's earlier LDS reads are done
#pragma unroll 1
  for (int j = 0; j < kw; ++j)  // word j of every lane's window -> ml[j * 64 + lane] (a lane past its window re-reads
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(mw + ((uint32_t)j < kl ? (uint32_t)j : kl - 1)),
                                     (__attribute__((address_space(3))) void*)(ml + j * 64), 4, 0, 0);  // its last)
  uint32_t Rw[8], Sw[8], Aw[8];
  int ok;
#ifdef AT2V_COMB_PROBE
  unsigned long long dummy = 0;
  unsigned long long& p_rec = pr ? pr->v[kCpRecord] : dummy;
  (void)p_rec;
#endif
  AT2V_CPROBE(p_rec, {
    load8(Rw, sig + (size_t)ii * 64);
    load8(Sw, sig + (size_t)ii * 64 + 32);
    load8(Aw, pk + (size_t)ii * 32);
    ok = comb_prechecks(Rw, Aw, Sw, policy, a_ok);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the staged message words have landed
  });
  const uint32_t msh = (o0 & 3u) * 8;
  auto staged = [=](uint32_t j) -> uint32_t {
    return __builtin_amdgcn_alignbit(ml[(j + 1) * 64 + lane], ml[j * 64 + lane], msh);
  };
  const DevComb tc{comb_key, {sa, sr}, lane};
#ifdef AT2V_COMB_PROBE
  if (pr) {
    uint32_t kd[kCombDigitWords], sd[BCombGeom<TabBC::kBits>::kDigitWords];
    AT2V_CPROBE(pr->v[kCpSha], {
      comb_k_digits(kd, Rw, Aw, len, staged);
      bcomb_recode<TabBC::kBits>(sd, Sw);
    });
    AT2V_CPROBE(pr->v[kCpSums], {
      gu_p3_identity(P);
      comb_sum<true>(P, kd, 0, kCombPos, tc);
      comb_sum<false>(P, sd, 0, BCombGeom<TabBC::kBits>::kPos, tbc);
    });
    pr->v[kCpAWait] += tc.waited;
    pr->v[kCpStage] += tc.stage_waited;
    pr->v[kCpLds] += tc.lds_waited;
    return ok;
  }
#endif
  comb_point(P, Rw, Aw, Sw, len, staged, tc, tbc);
  return ok;
}

// Comb throughput path with two records per lane (at2v_opts.sender_comb): a chunk is 128 records, lane l
// verifies records 128c + l and 128c + 64 + l. If all 128 hit the cache, both R' come from comb additions and their two
// inversions share one (Montgomery's trick: 1/Z0 = Z1 / (Z0 Z1), 1/Z1 = Z0 / (Z0 Z1)); otherwise each 64-record half runs
// the uncached half-size path. Chunks come from the per-launch queue as in verify_chunks.
__device__ AT2V_INLINE void verify_chunks_comb2(
    int4* astage, int4* rstage, const uint8_t* __restrict__ pk, const uint8_t* __restrict__ sig,
    const uint8_t* __restrict__ msg, uint32_t msg_total, const uint32_t* __restrict__ off, uint32_t n, int policy,
    uint32_t* __restrict__ verdicts, int4* __restrict__ scratch, const int4* __restrict__ btab,
    uint32_t* __restrict__ chunk_queue, const CacheArgs& cc) {
  const int lane = threadIdx.x & 63;
  const int wib = AT2V_UNIFORM(threadIdx.x >> 6);
  const uint32_t wave = blockIdx.x * kWavesPerBlock + wib;
  const uint32_t nwaves = gridDim.x * kWavesPerBlock;
  const uint32_t nchunks = (n + 127) / 128;
  const int4* __restrict__ comb = cc.payload;
  const uint32_t nwords = (n + 31) / 32;
  int4* slot = scratch + ((size_t)wave * 64 + lane) * kLaneGranules;
  const int4* ident = btab + (size_t)kNumBtabs * kBtabEntries * 8;
  int4* const sa = astage + wib * 640;
  int4* const sr = rstage + wib * 640;
  DevTabA ta{slot, sa, lane, ident};
  DevTabA tr{slot + kTabAGranules, sr, lane, ident};
  const DevTabB tb0{btab, sa, lane};
  const DevTabB tb1{btab + (size_t)kBtabEntries * 8, sr, lane};
  const DevBCombLat tbc{cc.bcomb_lat, {sa, sr}, lane};
  auto wmax = [](int v) { return wave_max_i32(v); };
  constexpr uint32_t kHalf = kWavesPerBlock / 2;
  const uint32_t c_first = wib < (int)kHalf ? blockIdx.x * kHalf + wib
                                            : gridDim.x * kHalf + blockIdx.x * kHalf + (wib - kHalf);
  for (uint32_t c = c_first; c < nchunks;) {
    // the cache check of both halves keeps only each record's hit, A-decode verdict and comb index; the records' words
    // are re-read where they are used, so at most one record's words and the other's R' are live at a time
    const uint32_t i0 = c * 128 + lane, i1 = i0 + 64;
    int a_ok0, a_ok1, cidx0, cidx1;
    int hit;
    {  // both halves' senders looked up (new keys claimed for the build stream) in the chunk prologue
      uint32_t Aw[8];
      load8(Aw, pk + (size_t)(i0 < n ? i0 : n - 1) * 32);
      hit = cache_hit(cc, cache_lookup_wave(cc, Aw, lane, i0 < n), Aw, a_ok0, cidx0) ? 1 : 0;
      load8(Aw, pk + (size_t)(i1 < n ? i1 : n - 1) * 32);
      hit &= cache_hit(cc, cache_lookup_wave(cc, Aw, lane, i1 < n), Aw, a_ok1, cidx1) ? 1 : 0;
    }
    const int all_hit = __builtin_amdgcn_readfirstlane(__all(hit) ? 1 : 0);
    if (lane == 0) {
      atomicAdd(cc.ctl + kCtlChunks, 2ull);
      if (all_hit) atomicAdd(cc.ctl + kCtlChunkHits, 2ull);
    }
    int good0, good1;
    if (all_hit) {
      gu_p3 P0, P1;
      const int ok0 = comb2_point(P0, i0, n, pk, sig, msg, msg_total, off, policy, a_ok0,
                                  comb + (size_t)cidx0 * (kCombBytes / 16), tbc, sa, sr, lane);
      const int ok1 = comb2_point(P1, i1, n, pk, sig, msg, msg_total, off, policy, a_ok1,
                                  comb + (size_t)cidx1 * (kCombBytes / 16), tbc, sa, sr, lane);
      fu zz, inv, zi;
      fu_mulc(zz, P0.Z, P1.Z);
      fu_invert(inv, zz);
      uint32_t Rw[8];
      load8(Rw, sig + (size_t)(i0 < n ? i0 : n - 1) * 64);
      fu_mulc(zi, inv, P1.Z);
      good0 = ok0 & gu_encode_eq_zi(P0, zi, Rw);
      load8(Rw, sig + (size_t)(i1 < n ? i1 : n - 1) * 64);
      fu_mulc(zi, inv, P0.Z);
      good1 = ok1 & gu_encode_eq_zi(P1, zi, Rw);
    } else {
      // one half at a time through ONE inlined copy of the ladder
      int g[2] = {0, 0};
#pragma unroll 1
      for (int h = 0; h < 2; ++h) {
        const uint32_t ii = h ? (i1 < n ? i1 : n - 1) : (i0 < n ? i0 : n - 1);
        uint32_t Rw[8], Sw[8], Aw[8];
        load8(Rw, sig + (size_t)ii * 64);
        load8(Sw, sig + (size_t)ii * 64 + 32);
        load8(Aw, pk + (size_t)ii * 32);
        const uint32_t o0 = off[ii], len = off[ii + 1] - o0;
        const int gh = with_msg_reader(msg, msg_total, o0, len, [&](auto& mwd) {
          return verify_half_fu(Rw, Aw, Sw, len, mwd, policy, ta, tr, tb0, tb1, wmax);
        });
        if (h) g[1] = gh;
        else g[0] = gh;
      }
      good0 = g[0];
      good1 = g[1];
    }
    const uint64_t m0 = __ballot(good0 & (i0 < n)), m1 = __ballot(good1 & (i1 < n));
    if (lane == 0) {
      const uint32_t w0 = 4 * c;
      if (w0 < nwords) verdicts[w0] = (uint32_t)m0;
      if (w0 + 1 < nwords) verdicts[w0 + 1] = (uint32_t)(m0 >> 32);
      if (w0 + 2 < nwords) verdicts[w0 + 2] = (uint32_t)m1;
      if (w0 + 3 < nwords) verdicts[w0 + 3] = (uint32_t)(m1 >> 32);
    }
    uint32_t ticket = 0;
    if (lane == 0) ticket = atomicAdd(chunk_queue, 1u);
    ticket = __builtin_amdgcn_readfirstlane(ticket);
    c = ticket < nchunks ? nwaves + ticket : nchunks;
  }
}

// Four records per lane (AT2V_COMB_PAIRS = 2): a chunk is 256 records, lane l verifies 256c + l + 64q, q = 0..3. All-hit
// chunks share ONE inversion among the four R' (Montgomery's trick over Z0 Z1 Z2 Z3): 63.5 S + 5 M per record instead of
// 127 S + 7 M with two records per lane (~9% of the comb path's multiplications). R'0 and R'1 are parked (X, Y, Z) in the
// lane's scratch slot while R'2 and R'3 are summed, and reloaded for their encodings. Other chunks run the four quarters
// through the half-size ladder.
// kPart: the chunks are 256 entries of the classify kernel's hit list (every record cached), verdict bits set by atomic
// OR; no ladder branch.
template <bool kPart = false>
#ifndef AT2V_COMB4_LOOP
#define AT2V_COMB4_LOOP 1  // the four records of a lane through one copy of the per-record code (0: four unrolled copies)
#endif
__device__ AT2V_INLINE void verify_chunks_comb4(
    int4* astage, int4* rstage, const uint8_t* __restrict__ pk, const uint8_t* __restrict__ sig,
    const uint8_t* __restrict__ msg, uint32_t msg_total, const uint32_t* __restrict__ off, uint32_t n, int policy,
    uint32_t* __restrict__ verdicts, int4* __restrict__ scratch, const int4* __restrict__ btab,
    uint32_t* __restrict__ chunk_queue, const CacheArgs& cc, const PartArgs* pp = nullptr) {
  const int lane = threadIdx.x & 63;
  const int wib = AT2V_UNIFORM(threadIdx.x >> 6);
  const uint32_t wave = blockIdx.x * kWavesPerBlock + wib;
  const uint32_t nwaves = gridDim.x * kWavesPerBlock;
  uint32_t nchunks = (n + 255) / 256, nh = 0;
  if constexpr (kPart) {
    nh = __builtin_amdgcn_readfirstlane(pp->counts[0]);
    nchunks = (nh + 255) / 256;
  }
  const int4* __restrict__ comb = cc.payload;
  const uint32_t nwords = (n + 31) / 32;
  int4* slot = scratch + ((size_t)wave * 64 + lane) * kLaneGranules;
  const int4* ident = btab + (size_t)kNumBtabs * kBtabEntries * 8;
  int4* const sa = astage + wib * 640;
  int4* const sr = rstage + wib * 640;
  DevTabA ta{slot, sa, lane, ident};
  DevTabA tr{slot + kTabAGranules, sr, lane, ident};
  const DevTabB tb0{btab, sa, lane};
  const DevTabB tb1{btab + (size_t)kBtabEntries * 8, sr, lane};
  const DevBCombLat tbc{cc.bcomb_lat, {sa, sr}, lane};
  auto wmax = [](int v) { return wave_max_i32(v); };
  constexpr uint32_t kHalf = kWavesPerBlock / 2;
  const uint32_t c_first = wib < (int)kHalf ? blockIdx.x * kHalf + wib
                                            : gridDim.x * kHalf + blockIdx.x * kHalf + (wib - kHalf);
  auto clamp = [n](uint32_t i) { return i < n ? i : n - 1; };
#ifdef AT2V_COMB_PROBE
  CombProbe probe;
  CombProbe* const pr = kPart ? &probe : nullptr;
#define AT2V_CP_ARG , pr
#else
#define AT2V_CP_ARG
#endif
  for (uint32_t c = c_first; c < nchunks;) {
#ifdef AT2V_COMB_PROBE
    const unsigned long long t_chunk0 = __builtin_amdgcn_s_memtime();
#endif
    const uint32_t i0 = c * 256 + lane;
    int a_ok[4], cidx[4];
    uint32_t rec[4];  // the four records of the lane
    int all_hit;
    if constexpr (kPart) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t pos = i0 + 64 * q, pc = pos < nh ? pos : nh - 1;
        rec[q] = pp->hidx[pc];
        const uint32_t info = pp->hinfo[pc];
        a_ok[q] = (int)(info & 1u);
        cidx[q] = (int)(info >> 1);
      }
#ifdef AT2V_COMB_PROBE
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the first use waits for them in the product build)
      probe.v[kCpBook] += __builtin_amdgcn_s_memtime() - t_chunk0;
#endif
      all_hit = 1;
    } else {
      int hit = 1;
#pragma unroll
      for (int q = 0; q < 4; ++q) {  // every quarter's sender looked up (new keys claimed for the build stream)
        uint32_t Aw[8];
        rec[q] = clamp(i0 + 64 * q);
        load8(Aw, pk + (size_t)rec[q] * 32);
        hit &= cache_hit(cc, cache_lookup_wave(cc, Aw, lane, i0 + 64 * q < n), Aw, a_ok[q], cidx[q]) ? 1 : 0;
      }
      all_hit = __builtin_amdgcn_readfirstlane(__all(hit) ? 1 : 0);
      if (lane == 0) {
        atomicAdd(cc.ctl + kCtlChunks, 4ull);
        if (all_hit) atomicAdd(cc.ctl + kCtlChunkHits, 4ull);
      }
    }
    const uint32_t lim = kPart ? nh : n;  // list / batch positions below lim are real
    int good[4] = {0, 0, 0, 0};
#if AT2V_COMB4_LOOP
    if (kPart || all_hit) {
      // ONE inlined copy of the per-record work, run four times: R'_q = comb sums of record q, parked in the slot (X, Y,
      // Z at granules 8q..8q+7). Four unrolled copies made the kernel 400 KB of code, whose hot loops (four copies of
      // SHA-512 and of the A and B comb loops) did not share the instruction cache between waves at different records.
      int okm = 0;
#pragma unroll 1
      for (int q = 0; q < 4; ++q) {
        const uint32_t rq = q == 0 ? rec[0] : q == 1 ? rec[1] : q == 2 ? rec[2] : rec[3];
        const int aq = q == 0 ? a_ok[0] : q == 1 ? a_ok[1] : q == 2 ? a_ok[2] : a_ok[3];
        const int cq = q == 0 ? cidx[0] : q == 1 ? cidx[1] : q == 2 ? cidx[2] : cidx[3];
        gu_p3 P;
        const int okq = comb2_point(P, rq, n, pk, sig, msg, msg_total, off, policy, aq,
                                    comb + (size_t)cq * (kCombBytes / 16), tbc, sa, sr, lane AT2V_CP_ARG);
        okm |= okq << q;
        slot_store(slot + 8 * q, reinterpret_cast<const int32_t*>(&P), 30);  // X, Y, Z (T not needed)
      }
#ifdef AT2V_COMB_PROBE
      const unsigned long long t_fin0 = __builtin_amdgcn_s_memtime();
#endif
      // Montgomery's trick: 1/Z_q = Z_{q^1} / (Z_q Z_{q^1}), and 1/(Z0 Z1), 1/(Z2 Z3) from one inversion
      fu inv01, inv23;
      {
        fu z0, z1, z2, z3, zz01, zz23, zz, inv;
        slot_load(reinterpret_cast<int32_t*>(z0.v), slot + 5, 10);
        slot_load(reinterpret_cast<int32_t*>(z1.v), slot + 8 + 5, 10);
        slot_load(reinterpret_cast<int32_t*>(z2.v), slot + 16 + 5, 10);
        slot_load(reinterpret_cast<int32_t*>(z3.v), slot + 24 + 5, 10);
        fu_mulc(zz01, z0, z1);
        fu_mulc(zz23, z2, z3);
        fu_mulc(zz, zz01, zz23);
        fu_invert(inv, zz);
        fu_mulc(inv01, inv, zz23);
        fu_mulc(inv23, inv, zz01);
      }
      int goodm = 0;
#pragma unroll 1
      for (int q = 0; q < 4; ++q) {
        const uint32_t rq = q == 0 ? rec[0] : q == 1 ? rec[1] : q == 2 ? rec[2] : rec[3];
        fu zp, zi;
        gu_p2 Q;
        slot_load(reinterpret_cast<int32_t*>(zp.v), slot + 8 * (q ^ 1) + 5, 10);  // the partner's Z
        slot_load(reinterpret_cast<int32_t*>(&Q), slot + 8 * q, 30);
        uint32_t Rw[8];
        load8(Rw, sig + (size_t)rq * 64);
        fu_mulc(zi, q < 2 ? inv01 : inv23, zp);
        goodm |= (((okm >> q) & 1) & gu_encode_eq_zi(Q, zi, Rw)) << q;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) good[q] = (goodm >> q) & 1;
#ifdef AT2V_COMB_PROBE
      probe.v[kCpFinish] += __builtin_amdgcn_s_memtime() - t_fin0;
#endif
    } else
#else
    if (kPart || all_hit) {
      int ok[4];
      fu zz01;
      {
        gu_p3 P0, P1;
        ok[0] = comb2_point(P0, rec[0], n, pk, sig, msg, msg_total, off, policy, a_ok[0],
                            comb + (size_t)cidx[0] * (kCombBytes / 16), tbc, sa, sr, lane AT2V_CP_ARG);
        ok[1] = comb2_point(P1, rec[1], n, pk, sig, msg, msg_total, off, policy, a_ok[1],
                            comb + (size_t)cidx[1] * (kCombBytes / 16), tbc, sa, sr, lane AT2V_CP_ARG);
        fu_mulc(zz01, P0.Z, P1.Z);
        slot_store(slot, reinterpret_cast<const int32_t*>(&P0), 30);        // X, Y, Z (T not needed)
        slot_store(slot + 8, reinterpret_cast<const int32_t*>(&P1), 30);
      }
      gu_p3 P2, P3;
      ok[2] = comb2_point(P2, rec[2], n, pk, sig, msg, msg_total, off, policy, a_ok[2],
                          comb + (size_t)cidx[2] * (kCombBytes / 16), tbc, sa, sr, lane AT2V_CP_ARG);
      ok[3] = comb2_point(P3, rec[3], n, pk, sig, msg, msg_total, off, policy, a_ok[3],
                          comb + (size_t)cidx[3] * (kCombBytes / 16), tbc, sa, sr, lane AT2V_CP_ARG);
#ifdef AT2V_COMB_PROBE
      const unsigned long long t_fin0 = __builtin_amdgcn_s_memtime();
#endif
      fu zz23, zz, inv, inv01, zi;
      fu_mulc(zz23, P2.Z, P3.Z);
      fu_mulc(zz, zz01, zz23);
      fu_invert(inv, zz);
      fu_mulc(inv01, inv, zz23);  // 1 / (Z0 Z1)
      fu_mulc(inv, inv, zz01);    // 1 / (Z2 Z3)
      uint32_t Rw[8];
      load8(Rw, sig + (size_t)rec[2] * 64);
      fu_mulc(zi, inv, P3.Z);
      good[2] = ok[2] & gu_encode_eq_zi(P2, zi, Rw);
      load8(Rw, sig + (size_t)rec[3] * 64);
      fu_mulc(zi, inv, P2.Z);
      good[3] = ok[3] & gu_encode_eq_zi(P3, zi, Rw);
      gu_p2 Q0, Q1;  // R'0 and R'1 back from the slot
      slot_load(reinterpret_cast<int32_t*>(&Q0), slot, 30);
      slot_load(reinterpret_cast<int32_t*>(&Q1), slot + 8, 30);
      load8(Rw, sig + (size_t)rec[0] * 64);
      fu_mulc(zi, inv01, Q1.Z);
      good[0] = ok[0] & gu_encode_eq_zi(Q0, zi, Rw);
      load8(Rw, sig + (size_t)rec[1] * 64);
      fu_mulc(zi, inv01, Q0.Z);
      good[1] = ok[1] & gu_encode_eq_zi(Q1, zi, Rw);
#ifdef AT2V_COMB_PROBE
      probe.v[kCpFinish] += __builtin_amdgcn_s_memtime() - t_fin0;
#endif
    } else
#endif  // AT2V_COMB4_LOOP
    {
      // one quarter at a time through ONE inlined copy of the ladder
#pragma unroll 1
      for (int q = 0; q < 4; ++q) {
        const uint32_t ii = clamp(i0 + 64 * q);  // (not kPart: the hit list never takes this branch)
        uint32_t Rw[8], Sw[8], Aw[8];
        load8(Rw, sig + (size_t)ii * 64);
        load8(Sw, sig + (size_t)ii * 64 + 32);
        load8(Aw, pk + (size_t)ii * 32);
        const uint32_t o0 = off[ii], len = off[ii + 1] - o0;
        const int gq = with_msg_reader(msg, msg_total, o0, len, [&](auto& mwd) {
          return verify_half_fu(Rw, Aw, Sw, len, mwd, policy, ta, tr, tb0, tb1, wmax);
        });
        good[0] = q == 0 ? gq : good[0];  // (selects, not a runtime index into a register array)
        good[1] = q == 1 ? gq : good[1];
        good[2] = q == 2 ? gq : good[2];
        good[3] = q == 3 ? gq : good[3];
      }
    }
#ifdef AT2V_COMB_PROBE
    const unsigned long long t_book0 = __builtin_amdgcn_s_memtime();
#endif
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if constexpr (kPart) {  // records in list order
        verdict_or(verdicts, rec[q], good[q], i0 + 64 * q < lim, lane);
      } else {
        const uint64_t m = __ballot(good[q] & (i0 + 64 * q < n));
        if (lane == 0) {
          const uint32_t w0 = 8 * c + 2 * q;
          if (w0 < nwords) verdicts[w0] = (uint32_t)m;
          if (w0 + 1 < nwords) verdicts[w0 + 1] = (uint32_t)(m >> 32);
        }
      }
    }
    uint32_t ticket = 0;
    if (lane == 0) ticket = atomicAdd(chunk_queue, 1u);
    ticket = __builtin_amdgcn_readfirstlane(ticket);
    c = ticket < nchunks ? nwaves + ticket : nchunks;
#ifdef AT2V_COMB_PROBE
    if constexpr (kPart) {
      const unsigned long long t_end = __builtin_amdgcn_s_memtime();
      probe.v[kCpBook] += t_end - t_book0;
      probe.v[kCpChunk] += t_end - t_chunk0;
      probe.v[kCpChunks] += 1;
      probe.v[kCpBWait] += tbc.waited;
      probe.v[kCpStage] += tbc.stage_waited;
      tbc.waited = tbc.stage_waited = 0;
    }
#endif
  }
#ifdef AT2V_COMB_PROBE
  if constexpr (kPart) {  // one vector atomic per counter and wave, from lane 0
    if (lane == 0)
#pragma unroll
      for (int k = 0; k < kCpN; ++k) atomicAdd(&at2v_cprobe_acc[k], probe.v[k]);
  }
#endif
#undef AT2V_CP_ARG
}

// the same with per-key combs (at2v_opts.sender_comb): all-hit waves verify by additions only
__global__ __launch_bounds__(kBlock, AT2V_VERIFY_WAVES_PER_SIMD) void verify_kernel_comb(
    const uint8_t* __restrict__ pk, const uint8_t* __restrict__ sig, const uint8_t* __restrict__ msg,
    uint32_t msg_total, const uint32_t* __restrict__ off, uint32_t n, int policy, uint32_t* __restrict__ verdicts,
    int4* __restrict__ scratch, const int4* __restrict__ btab, uint32_t* __restrict__ chunk_queue, CacheArgs c) {
  __shared__ int4 astage[kWavesPerBlock * 10 * 64];
  __shared__ int4 rstage[kWavesPerBlock * 10 * 64];
#ifndef AT2V_COMB_PAIRS
#define AT2V_COMB_PAIRS 2  // 1: two records per lane, one shared inversion (verify_chunks_comb2); 2: four
                           // (verify_chunks_comb4); 0: one record per lane
#endif
#if AT2V_COMB_PAIRS == 2
  verify_chunks_comb4<false>(astage, rstage, pk, sig, msg, msg_total, off, n, policy, verdicts, scratch, btab,
                             chunk_queue, c);
#elif AT2V_COMB_PAIRS
  verify_chunks_comb2(astage, rstage, pk, sig, msg, msg_total, off, n, policy, verdicts, scratch, btab, chunk_queue, c);
#else
  static_assert(AT2V_LADDER_BW == 16, "the one-record-per-lane comb kernel keeps the 16-bit fixed-base tables");
  verify_chunks<true, true>(astage, rstage, pk, sig, msg, msg_total, off, n, policy, verdicts, scratch, btab, btab,
                            chunk_queue, &c);
#endif
}

// The classify kernel's hit list by comb additions, kRecs records per lane (chunks of 64 kRecs list positions): each
// record's R' = [k](-A) + [s]B is parked in the lane's slot (X, Y, Z at granules 8q..8q+7), then ONE inversion serves
// all kRecs Z's (Montgomery's trick as a product tree: pair products zp, for 8 records quad products, the inverse of the
// product, back down to 1 / (Z_2k Z_2k+1) at granules 8 kRecs + 3k), and each record is encoded with
// 1 / Z_q = Z_{q^1} / (Z_q Z_{q^1}). Per record: 254/kRecs squarings of the inversion, (3 kRecs - 3)/kRecs + 2
// products. Verdict bits go to the record's place in the bitmap (verdict_or).
#ifndef AT2V_COMB_MSG_STAGE
#define AT2V_COMB_MSG_STAGE 1  // messages staged in LDS before SHA-512 (comb2_point_staged); 0: read word by word
#endif
template <int kRecs, int kBW, int kWaves = kWavesPerBlock>
__device__ AT2V_INLINE void verify_comb_hits(int4* astage, int4* rstage, const uint8_t* __restrict__ pk,
                                             const uint8_t* __restrict__ sig, const uint8_t* __restrict__ msg,
                                             uint32_t msg_total, const uint32_t* __restrict__ off, uint32_t n,
                                             int policy, uint32_t* __restrict__ verdicts, int4* __restrict__ scratch,
                                             uint32_t* __restrict__ chunk_queue, const CacheArgs& cc,
                                             const PartArgs& pp, uint32_t nh) {
  static_assert(kRecs == 4 || kRecs == 8, "records per lane");
  static_assert(8 * kRecs + 3 * (kRecs / 2) <= kLaneGranules, "the slot holds the parked points and pair inverses");
  const int lane = threadIdx.x & 63;
  const int wib = AT2V_UNIFORM(threadIdx.x >> 6);
  const uint32_t wave = blockIdx.x * kWaves + wib;
  const uint32_t nwaves = gridDim.x * kWaves;
  constexpr uint32_t kChunk = 64 * kRecs;
  const uint32_t nchunks = (nh + kChunk - 1) / kChunk;
  const int4* __restrict__ comb = cc.payload;
  int4* slot = scratch + ((size_t)wave * 64 + lane) * kLaneGranules;
  int4* const pinv = slot + 8 * kRecs;  // 1 / (Z_2k Z_2k+1), 3 granules each
  int4* const sa = astage + wib * 640;
  int4* const sr = rstage + wib * 640;
  // the context's wide comb of B (AT2V_CTX_BCOMB_WIDE, 24-bit windows: five additions fewer) or the 16-bit one
  const DevBCombW<kBW> tbc{kBW == kBCombLatBits ? cc.bcomb_lat : cc.bcomb, {sa, sr}, lane};
  constexpr uint32_t kHalf = kWaves / 2;
  const uint32_t c_first = wib < (int)kHalf ? blockIdx.x * kHalf + wib
                                            : gridDim.x * kHalf + blockIdx.x * kHalf + (wib - kHalf);
  auto zload = [&](fu& z, int q) { slot_load(reinterpret_cast<int32_t*>(z.v), slot + 8 * q + 5, 10); };
#ifdef AT2V_COMB_PROBE
  CombProbe probe;
  CombProbe* const pr = &probe;
#endif
  for (uint32_t c = c_first; c < nchunks;) {
#ifdef AT2V_COMB_PROBE
    const unsigned long long t_chunk0 = __builtin_amdgcn_s_memtime();
#endif
    const uint32_t i0 = c * kChunk + lane;
#if AT2V_COMB_MSG_STAGE
    // the chunk's list entries, then their records' offsets: two memory latencies per chunk, not per record
    uint32_t lrec[kRecs], linfo[kRecs], lo0[kRecs], llen[kRecs];
#pragma unroll
    for (int q = 0; q < kRecs; ++q) {
      const uint32_t pos = i0 + 64 * q, pc = pos < nh ? pos : nh - 1;
      lrec[q] = pp.hidx[pc];
      linfo[q] = pp.hinfo[pc];
    }
#pragma unroll
    for (int q = 0; q < kRecs; ++q) {
      lo0[q] = off[lrec[q]];
      llen[q] = off[lrec[q] + 1] - lo0[q];
    }
#endif
    int okm = 0;
#pragma unroll 1
    for (int q = 0; q < kRecs; ++q) {
#if AT2V_COMB_MSG_STAGE
      uint32_t rq = lrec[0], info = linfo[0], o0 = lo0[0], len = llen[0];
#pragma unroll
      for (int k = 1; k < kRecs; ++k)
        if (q == k) {  // (selects: a runtime index into a register array would go to scratch)
          rq = lrec[k];
          info = linfo[k];
          o0 = lo0[k];
          len = llen[k];
        }
#else
      const uint32_t pos = i0 + 64 * q, pc = pos < nh ? pos : nh - 1;
      const uint32_t rq = pp.hidx[pc], info = pp.hinfo[pc];
#endif
      gu_p3 P;
      int okq = -1;
#if AT2V_COMB_MSG_STAGE
      okq = comb2_point_staged(P, rq, o0, len, pk, sig, msg, msg_total, policy, (int)(info & 1u),
                               comb + (size_t)(info >> 1) * (kCombBytes / 16), tbc, sa, sr, lane
#ifdef AT2V_COMB_PROBE
                               , pr
#endif
      );
#endif
      if (okq < 0)
        okq = comb2_point(P, rq, n, pk, sig, msg, msg_total, off, policy, (int)(info & 1u),
                          comb + (size_t)(info >> 1) * (kCombBytes / 16), tbc, sa, sr, lane
#ifdef AT2V_COMB_PROBE
                          , pr
#endif
        );
      okm |= okq << q;
      slot_store(slot + 8 * q, reinterpret_cast<const int32_t*>(&P), 30);  // X, Y, Z (T not needed)
    }
#ifdef AT2V_COMB_PROBE
    const unsigned long long t_fin0 = __builtin_amdgcn_s_memtime();
#endif
    {
      fu z0, z1, zp0, zp1, inv;
      zload(z0, 0);
      zload(z1, 1);
#ifdef AT2V_COMB_PROBE
      AT2V_CPROBE(probe.v[kCpSlot], asm volatile("s_waitcnt vmcnt(0)" ::: "memory"));
#endif
      fu_mulc(zp0, z0, z1);
      zload(z0, 2);
      zload(z1, 3);
#ifdef AT2V_COMB_PROBE
      AT2V_CPROBE(probe.v[kCpSlot], asm volatile("s_waitcnt vmcnt(0)" ::: "memory"));
#endif
      fu_mulc(zp1, z0, z1);
      if constexpr (kRecs == 4) {
        fu_mulc(z0, zp0, zp1);
        fu_invert(inv, z0);
        fu_mulc(z0, inv, zp1);  // 1 / (Z0 Z1)
        slot_store(pinv, reinterpret_cast<const int32_t*>(z0.v), 10);
        fu_mulc(z0, inv, zp0);  // 1 / (Z2 Z3)
        slot_store(pinv + 3, reinterpret_cast<const int32_t*>(z0.v), 10);
      } else {
        fu zp2, zp3, zq0, zq1;
        zload(z0, 4);
        zload(z1, 5);
        fu_mulc(zp2, z0, z1);
        zload(z0, 6);
        zload(z1, 7);
        fu_mulc(zp3, z0, z1);
        fu_mulc(zq0, zp0, zp1);
        fu_mulc(zq1, zp2, zp3);
        fu_mulc(z0, zq0, zq1);
        fu_invert(inv, z0);
        fu_mulc(z0, inv, zq1);  // 1 / (Z0 Z1 Z2 Z3)
        fu_mulc(z1, z0, zp1);   // 1 / (Z0 Z1)
        slot_store(pinv, reinterpret_cast<const int32_t*>(z1.v), 10);
        fu_mulc(z1, z0, zp0);   // 1 / (Z2 Z3)
        slot_store(pinv + 3, reinterpret_cast<const int32_t*>(z1.v), 10);
        fu_mulc(z0, inv, zq0);  // 1 / (Z4 Z5 Z6 Z7)
        fu_mulc(z1, z0, zp3);   // 1 / (Z4 Z5)
        slot_store(pinv + 6, reinterpret_cast<const int32_t*>(z1.v), 10);
        fu_mulc(z1, z0, zp2);   // 1 / (Z6 Z7)
        slot_store(pinv + 9, reinterpret_cast<const int32_t*>(z1.v), 10);
      }
    }
#pragma unroll 1
    for (int q = 0; q < kRecs; ++q) {
      const uint32_t pos = i0 + 64 * q, pc = pos < nh ? pos : nh - 1;
      const uint32_t rq = pp.hidx[pc];
      fu zp, ip, zi;
      gu_p2 Q;
      zload(zp, q ^ 1);  // the partner's Z
      slot_load(reinterpret_cast<int32_t*>(ip.v), pinv + 3 * (q >> 1), 10);
      slot_load(reinterpret_cast<int32_t*>(&Q), slot + 8 * q, 30);
      uint32_t Rw[8];
      load8(Rw, sig + (size_t)rq * 64);
#ifdef AT2V_COMB_PROBE
      AT2V_CPROBE(probe.v[kCpSlot], asm volatile("s_waitcnt vmcnt(0)" ::: "memory"));
#endif
      fu_mulc(zi, ip, zp);
      const int good = ((okm >> q) & 1) & gu_encode_eq_zi(Q, zi, Rw);
      verdict_or(verdicts, rq, good, pos < nh, lane);
    }
#ifdef AT2V_COMB_PROBE
    const unsigned long long t_book0 = __builtin_amdgcn_s_memtime();
    probe.v[kCpFinish] += t_book0 - t_fin0;
#endif
    uint32_t ticket = 0;
    if (lane == 0) ticket = atomicAdd(chunk_queue, 1u);
    ticket = __builtin_amdgcn_readfirstlane(ticket);
    c = ticket < nchunks ? nwaves + ticket : nchunks;
#ifdef AT2V_COMB_PROBE
    const unsigned long long t_end = __builtin_amdgcn_s_memtime();
    probe.v[kCpBook] += t_end - t_book0;
    probe.v[kCpChunk] += t_end - t_chunk0;
    probe.v[kCpChunks] += 1;
    probe.v[kCpBWait] += tbc.waited;
    probe.v[kCpStage] += tbc.stage_waited;
    probe.v[kCpLds] += tbc.lds_waited;
    tbc.waited = tbc.stage_waited = tbc.lds_waited = 0;
#endif
  }
#ifdef AT2V_COMB_PROBE
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < kCpN; ++k) atomicAdd(&at2v_cprobe_acc[k], probe.v[k]);
#endif
}

// partitioned cached launches: the classify kernel's hit list by comb additions, four records per lane (eight per lane,
// one inversion for eight, measured 1.4% slower on 1M records from 64 senders: one 512-record chunk per wave leaves
// the chunk queue nothing to balance, profiles/r05n/abcomb.txt), [s]B from the context's 20-bit or 24-bit comb of B
__global__ __launch_bounds__(kBlock, AT2V_VERIFY_WAVES_PER_SIMD) void verify_kernel_comb_part(
    const uint8_t* __restrict__ pk, const uint8_t* __restrict__ sig, const uint8_t* __restrict__ msg,
    uint32_t msg_total, const uint32_t* __restrict__ off, uint32_t n, int policy, uint32_t* __restrict__ verdicts,
    int4* __restrict__ scratch, const int4* __restrict__ btab, uint32_t* __restrict__ chunk_queue, CacheArgs c,
    PartArgs p) {
  __shared__ int4 astage[kWavesPerBlock * 10 * 64];
  __shared__ int4 rstage[kWavesPerBlock * 10 * 64];
  (void)btab;
  const uint32_t nh = __builtin_amdgcn_readfirstlane(p.counts[0]);
  if (c.bcomb_bits == kBCombBits)  // AT2V_CTX_BCOMB_WIDE
    verify_comb_hits<4, kBCombBits>(astage, rstage, pk, sig, msg, msg_total, off, n, policy, verdicts, scratch,
                                    chunk_queue, c, p, nh);
  else
    verify_comb_hits<4, kBCombMidBits>(astage, rstage, pk, sig, msg, msg_total, off, n, policy, verdicts, scratch,
                                       chunk_queue, c, p, nh);
}

#if AT2V_EXP_COMB3
__global__ __launch_bounds__(768, 3) void verify_kernel_comb_part3(
    const uint8_t* __restrict__ pk, const uint8_t* __restrict__ sig, const uint8_t* __restrict__ msg,
    uint32_t msg_total, const uint32_t* __restrict__ off, uint32_t n, int policy, uint32_t* __restrict__ verdicts,
    int4* __restrict__ scratch, uint32_t* __restrict__ chunk_queue, CacheArgs c, PartArgs p) {
  __shared__ int4 stage[12 * 10 * 64];
  const uint32_t nh = __builtin_amdgcn_readfirstlane(p.counts[0]);
  if (c.bcomb_bits == kBCombBits)
    verify_comb_hits<4, kBCombBits, 12>(stage, stage, pk, sig, msg, msg_total, off, n, policy, verdicts, scratch,
                                        chunk_queue, c, p, nh);
  else
    verify_comb_hits<4, kBCombMidBits, 12>(stage, stage, pk, sig, msg, msg_total, off, n, policy, verdicts, scratch,
                                           chunk_queue, c, p, nh);
}
#endif

// ---------------------------------------------------------------------------------------------------------------
// Low-latency verify for small launches: two lanes per record (lane 2r: A side, lane 2r+1: R side,
// verify_pair_part), 32 records per wave, one wave per SIMD (4-wave blocks, 80 KiB LDS). Each lane decodes one point,
// builds one table and does one addition per window; the partner's cached point comes across by __shfl_xor and both
// lanes evaluate V = P0 + P1 (verify_pair_combine). Chunks c = 32-record groups, grid-strided.
constexpr int kPairBlock = 256;
constexpr int kPairWaves = kPairBlock / 64;
__global__ __launch_bounds__(kPairBlock, 1) void verify_pair_kernel(
    const uint8_t* __restrict__ pk, const uint8_t* __restrict__ sig, const uint8_t* __restrict__ msg,
    uint32_t msg_total, const uint32_t* __restrict__ off, uint32_t n, int policy, uint32_t* __restrict__ verdicts,
    int4* __restrict__ scratch, const int4* __restrict__ btab) {
  __shared__ int4 pstage[kPairWaves * 10 * 64];
  __shared__ int4 bstage[kPairWaves * 10 * 64];
  const int lane = threadIdx.x & 63;
  const int wib = AT2V_UNIFORM(threadIdx.x >> 6);  // wave-uniform: the LDS stage addresses live in SGPRs
  const int side = lane & 1;
  const uint32_t wave = blockIdx.x * kPairWaves + wib;
  const uint32_t nwaves = gridDim.x * kPairWaves;
  const uint32_t nchunks = (n + 31) / 32;
  int4* slot = scratch + ((size_t)wave * 64 + lane) * kTabAGranules;
  DevTabA tp{slot, pstage + wib * 640, lane, btab + (size_t)kNumBtabs * kBtabEntries * 8};
  const DevTabB tb{btab + (size_t)side * kBtabEntries * 8, bstage + wib * 640, lane};
  auto wmax = [](int v) { return wave_max_i32(v); };
  for (uint32_t c = wave; c < nchunks; c += nwaves) {
    const uint32_t i = c * 32 + (lane >> 1);
    const uint32_t ii = i < n ? i : n - 1;  // tail lanes recompute a real record; their bit is masked
    uint32_t Rw[8], Sw[8], Aw[8];
    load8(Rw, sig + (size_t)ii * 64);
    load8(Sw, sig + (size_t)ii * 64 + 32);
    load8(Aw, pk + (size_t)ii * 32);
    const uint32_t o0 = off[ii];
    const uint32_t len = off[ii + 1] - o0;
    const int msg_fast =
        __builtin_amdgcn_readfirstlane(__all((uint64_t)o0 + len + 8 <= (uint64_t)msg_total) ? 1 : 0);
    const uint32_t* mw = reinterpret_cast<const uint32_t*>(msg) + (o0 >> 2);
    const uint32_t msh = (o0 & 3u) * 8;
    auto msgword = [&](uint32_t j) -> uint32_t {
      if (msg_fast) return __builtin_amdgcn_alignbit(mw[j + 1], mw[j], msh);
      const uint32_t a = o0 + 4 * j;
      const uint32_t a0 = a & ~3u, sh = (a & 3u) * 8;
      const uint32_t lo = load_u32_guarded(msg, a0, msg_total);
      if (sh == 0) return lo;
      const uint32_t hi = load_u32_guarded(msg, a0 + 4, msg_total);
      return __builtin_amdgcn_alignbit(hi, lo, sh);
    };
    gu_p3 Pm;
    int ok = verify_pair_part(side, Rw, Aw, Sw, len, msgword, policy, tp, tb, wmax, Pm);
    gu_cached cm, cp;
    gu_p3_to_cached(cm, Pm);
    const uint32_t* cw = reinterpret_cast<const uint32_t*>(&cm);
    uint32_t* pw = reinterpret_cast<uint32_t*>(&cp);
#pragma unroll
    for (int q = 0; q < 40; ++q) pw[q] = (uint32_t)__shfl_xor((int)cw[q], 1);
    ok &= __shfl_xor(ok, 1);
    const int good = ok & verify_pair_combine(Pm, cp) & (i < n);
    const uint64_t mask = __ballot(good);
    if (lane == 0) {  // record r's verdict is lane 2r's bit: compress the even bits of the ballot
      uint64_t x = mask & 0x5555555555555555ull;
      x = (x | (x >> 1)) & 0x3333333333333333ull;
      x = (x | (x >> 2)) & 0x0f0f0f0f0f0f0f0full;
      x = (x | (x >> 4)) & 0x00ff00ff00ff00ffull;
      x = (x | (x >> 8)) & 0x0000ffff0000ffffull;
      x = (x | (x >> 16)) & 0x00000000ffffffffull;
      verdicts[c] = (uint32_t)x;
    }
  }
}
#else
__global__ __launch_bounds__(kBlock, AT2V_VERIFY_WAVES_PER_SIMD) void verify_kernel(
    const uint8_t* __restrict__ pk, const uint8_t* __restrict__ sig, const uint8_t* __restrict__ msg,
    uint32_t msg_total, const uint32_t* __restrict__ off, uint32_t n, int policy, uint32_t* __restrict__ verdicts,
    int4* __restrict__ scratch, const int4* __restrict__ btab, const int4* __restrict__ btab24,
    uint32_t* __restrict__ chunk_queue) {
  __shared__ int4 astage[kWavesPerBlock * 10 * 64];
  __shared__ int4 bstage[kWavesPerBlock * 8 * 64];
  const int lane = threadIdx.x & 63;
  const uint32_t wave = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  const uint32_t nwaves = gridDim.x * kWavesPerBlock;
  const uint32_t nchunks = (n + 63) / 64;
  const uint32_t nwords = (n + 31) / 32;
  int4* slot = scratch + ((size_t)wave * 64 + lane) * kLaneGranules;
  DevTabA ta{slot, astage + (threadIdx.x >> 6) * 640, lane};
  DevTabB tb{btab, bstage + (threadIdx.x >> 6) * 512, lane};
  int4* park = slot + kTabAGranules;                 // kGroup x 8 granules: R' of chunk h of the group
  int4* pref = slot + kTabAGranules + kParkGranules;  // (kGroup-1) x 3 granules: Z_0 * .. * Z_h
  // Chunks are taken in groups (c, c + nwaves, ..., c + (kGroup-1) nwaves): one field inversion serves the
  // whole group (Montgomery's trick, 3 M per extra chunk). The ladder body appears once (rolled loop).
  for (uint32_t c = wave; c < nchunks; c += kGroup * nwaves) {
    const int cnt = (int)min((uint32_t)kGroup, (nchunks - c + nwaves - 1) / nwaves);
    uint32_t okbits = 0;
    AT2V_PHASE(0);
#pragma unroll 1
    for (int h = 0; h < cnt; ++h) {
      const uint32_t chunk = c + (uint32_t)h * nwaves;
      const uint32_t i = chunk * 64 + lane;
      const uint32_t ii = i < n ? i : n - 1;  // tail lanes recompute a real record; their bit is masked
      uint32_t Rw[8], Sw[8], Aw[8];
      load8(Rw, sig + (size_t)ii * 64);
      load8(Sw, sig + (size_t)ii * 64 + 32);
      load8(Aw, pk + (size_t)ii * 32);
      const uint32_t o0 = off[ii];
      const uint32_t len = off[ii + 1] - o0;
      auto msgword = [&](uint32_t j) -> uint32_t {
        const uint32_t a = o0 + 4 * j;
        const uint32_t a0 = a & ~3u, sh = (a & 3u) * 8;
        const uint32_t lo = load_u32_guarded(msg, a0, msg_total);
        if (sh == 0) return lo;
        const uint32_t hi = load_u32_guarded(msg, a0 + 4, msg_total);
        return __builtin_amdgcn_alignbit(hi, lo, sh);
      };
      ge_p2 Rp;
      const int ok = verify_ladder<kBWin>(Rp, Rw, Aw, Sw, len, msgword, policy, ta, tb) & (i < n);
      okbits |= (uint32_t)ok << h;
      slot_store(park + 8 * h, reinterpret_cast<const int32_t*>(&Rp), 30);
    }
    // prefix products P_h = Z_0 ... Z_h (P_0..P_{cnt-2} kept in scratch), one inversion of P_{cnt-1}
    fe acc;
    slot_load(acc.v, park + 5, 10);  // Z of chunk 0 (words 20..29 of the parked point)
#pragma unroll 1
    for (int h = 1; h < cnt; ++h) {
      slot_store(pref + 3 * (h - 1), acc.v, 10);
      fe z;
      slot_load(z.v, park + 8 * h + 5, 10);
      fe_mul(acc, acc, z);
    }
    fe inv;
    fe_invert(inv, acc);
    AT2V_PHASE(5);
    // backwards: 1/Z_h = inv_h * P_{h-1} with inv_h = 1/P_h; inv_{h-1} = inv_h * Z_h
#pragma unroll 1
    for (int h = cnt - 1; h >= 0; --h) {
      ge_p2 R;
      slot_load(reinterpret_cast<int32_t*>(&R), park + 8 * h, 30);
      fe zi;
      if (h > 0) {
        fe p;
        slot_load(p.v, pref + 3 * (h - 1), 10);
        fe_mul(zi, inv, p);
        fe_mul(inv, inv, R.Z);
      } else {
        zi = inv;
      }
      const uint32_t chunk = c + (uint32_t)h * nwaves;
      const uint32_t i = chunk * 64 + lane;
      const uint32_t ii = i < n ? i : n - 1;
      uint32_t Rr[8];
      load8(Rr, sig + (size_t)ii * 64);
      const int good = (int)((okbits >> h) & 1u) & verify_finish(R, zi, Rr);
      const uint64_t mask = __ballot(good);
      if (lane == 0) {
        verdicts[2 * chunk] = (uint32_t)mask;
        if (2 * chunk + 1 < nwords) verdicts[2 * chunk + 1] = (uint32_t)(mask >> 32);
      }
    }
    AT2V_PHASE(6);
  }
}

#endif  // AT2V_VERIFY_HALF

// ------------------------------------------------------------------ signing side

__device__ AT2V_INLINE void sc_muladd(uint32_t out[8], const uint32_t a[8], const uint32_t b[8], const uint32_t c[8]) {
  uint32_t x[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint64_t t = (uint64_t)a[i] * b[j] + x[i + j] + carry;
      x[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    x[i + 8] = (uint32_t)carry;
  }
  uint64_t carry = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const uint64_t t = (uint64_t)x[i] + (i < 8 ? c[i] : 0u) + carry;
    x[i] = (uint32_t)t;
    carry = t >> 32;
  }
  sc_reduce512(out, x);  // a, b, c < 2^253 so the sum < 2^507
}

// RFC 8032 sign of M under `seed` (8 LE words); writes pk (8 words) and R||S (16 words)
template <class TabB, class MsgWord>
__device__ AT2V_INLINE void sign_core(uint32_t pkw[8], uint32_t sigw[16], const uint32_t seed[8], uint32_t len,
                                      MsgWord msgword, const TabB& tb) {
  uint64_t h[8];
  uint32_t hw[16];
  sha512_prefixed<8>(h, seed, 0, [](uint32_t) { return 0u; });
  sha512_digest_words(hw, h);
  uint32_t a[8], prefix[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a[i] = hw[i];
    prefix[i] = hw[8 + i];
  }
  a[0] &= 0xfffffff8u;
  a[7] = (a[7] & 0x7fffffffu) | 0x40000000u;
  uint32_t a16[16], ared[8];
#pragma unroll
  for (int i = 0; i < 16; ++i) a16[i] = i < 8 ? a[i] : 0u;
  sc_reduce512(ared, a16);
  ge_p2 P;
  ge_scalarmult_base(P, ared, tb);
  ge_p2_tobytes(pkw, P);
  // r = H(prefix || M) mod l ; R = [r]B
  sha512_prefixed<8>(h, prefix, len, msgword);
  sha512_digest_words(hw, h);
  uint32_t r[8];
  sc_reduce512(r, hw);
  ge_scalarmult_base(P, r, tb);
  ge_p2_tobytes(sigw, P);
  // k = H(R || A || M) mod l ; S = r + k a mod l
  uint32_t pre[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    pre[i] = sigw[i];
    pre[8 + i] = pkw[i];
  }
  sha512_prefixed<16>(h, pre, len, msgword);
  sha512_digest_words(hw, h);
  uint32_t k[8];
  sc_reduce512(k, hw);
  sc_muladd(sigw + 8, k, ared, r);
}

// SHA-512 of a short byte string held in registers as LE words (len <= 64)
template <int NW>
__device__ AT2V_INLINE void sha512_words(uint32_t out16[16], const uint32_t (&wds)[NW], uint32_t len) {
  uint64_t h[8];
  sha512_prefixed<0>(h, nullptr, len, [&](uint32_t j) {
    uint32_t v = 0;
#pragma unroll
    for (int m = 0; m < NW; ++m) v = (j == (uint32_t)m) ? wds[m] : v;
    return v;
  });
  sha512_digest_words(out16, h);
}

// seed_i and M_i of the deterministic generator (byte strings "at2v/seed"||u64le||u64le, 25 bytes, and
// "at2v/msg"||u64le cfg||u64le i||u64le ctr, 32 bytes)
__device__ AT2V_INLINE void gen_seed(uint32_t seed[8], uint64_t cfg, uint64_t idx) {
  // bytes: a t 2 v / s e e d | cfg(8) | idx(8)
  uint32_t w[7];
  w[0] = 0x76327461u;                                               // "at2v"
  w[1] = 0x6565732fu;                                               // "/see"
  w[2] = 0x64u | ((uint32_t)(cfg & 0xffffff) << 8);                 // "d" + cfg[0..2]
  w[3] = (uint32_t)(cfg >> 24);                                     // cfg[3..6]
  w[4] = (uint32_t)(cfg >> 56) | ((uint32_t)(idx & 0xffffff) << 8); // cfg[7] + idx[0..2]
  w[5] = (uint32_t)(idx >> 24);                                     // idx[3..6]
  w[6] = (uint32_t)(idx >> 56);                                     // idx[7]
  uint32_t o[16];
  sha512_words<7>(o, w, 25);
#pragma unroll
  for (int i = 0; i < 8; ++i) seed[i] = o[i];
}

__device__ AT2V_INLINE void gen_msg_block(uint32_t out16[16], uint64_t cfg, uint64_t idx, uint64_t ctr) {
  uint32_t w[8];
  w[0] = 0x76327461u;  // "at2v"
  w[1] = 0x67736d2fu;  // "/msg"
  w[2] = (uint32_t)cfg;
  w[3] = (uint32_t)(cfg >> 32);
  w[4] = (uint32_t)idx;
  w[5] = (uint32_t)(idx >> 32);
  w[6] = (uint32_t)ctr;
  w[7] = (uint32_t)(ctr >> 32);
  sha512_words<8>(out16, w, 32);
}

__global__ __launch_bounds__(kBlock) void gen_kernel(uint64_t cfg, uint64_t first, uint32_t n, uint32_t msg_len,
                                                     uint64_t senders, const uint64_t* __restrict__ keys,
                                                     uint8_t* __restrict__ pk,
                                                     uint8_t* __restrict__ sig, uint8_t* __restrict__ msg,
                                                     uint32_t* __restrict__ off) {
  __shared__ int4 btab[AT2V_BTAB_ENTRIES * 8];
  stage_btab(btab);
  LdsTabB tb{btab};
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t idx = first + i;
  uint32_t seed[8];
  // the key of seed index keys[i] (at2v_gen_records_keys_device), or of sender idx % senders; M_i stays per record
  gen_seed(seed, cfg, keys ? keys[i] : senders ? idx % senders : idx);
  // message bytes into the output buffer (byte stores; msg_len arbitrary)
  uint8_t* m = msg + (size_t)i * msg_len;
  for (uint32_t ctr = 0; ctr * 64 < msg_len; ++ctr) {
    uint32_t blk[16];
    gen_msg_block(blk, cfg, idx, ctr);
    for (uint32_t b = 0; b < 64 && ctr * 64 + b < msg_len; ++b) m[ctr * 64 + b] = (uint8_t)(blk[b >> 2] >> (8 * (b & 3)));
  }
  if (off) {
    off[i] = i * msg_len;
    if (i == n - 1) off[n] = n * msg_len;
  }
  const uint32_t mtotal = n * msg_len, o0 = i * msg_len;
  auto msgword = [&](uint32_t j) -> uint32_t {  // this lane's own bytes, written just above
    const uint32_t a = o0 + 4 * j;
    const uint32_t a0 = a & ~3u, sh = (a & 3u) * 8;
    const uint32_t lo = load_u32_guarded(msg, a0, mtotal);
    if (sh == 0) return lo;
    return __builtin_amdgcn_alignbit(load_u32_guarded(msg, a0 + 4, mtotal), lo, sh);
  };
  uint32_t pkw[8], sigw[16];
  sign_core(pkw, sigw, seed, msg_len, msgword, tb);
  uint32_t* pko = reinterpret_cast<uint32_t*>(pk + (size_t)i * 32);
  uint32_t* sgo = reinterpret_cast<uint32_t*>(sig + (size_t)i * 64);
#pragma unroll
  for (int q = 0; q < 8; ++q) pko[q] = pkw[q];
#pragma unroll
  for (int q = 0; q < 16; ++q) sgo[q] = sigw[q];
}

__global__ __launch_bounds__(kBlock) void sign_kernel(const uint8_t* __restrict__ seeds, const uint8_t* __restrict__ msg,
                                                      uint32_t msg_total, const uint32_t* __restrict__ off, uint32_t n,
                                                      uint8_t* __restrict__ pk, uint8_t* __restrict__ sig) {
  __shared__ int4 btab[AT2V_BTAB_ENTRIES * 8];
  stage_btab(btab);
  LdsTabB tb{btab};
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t seed[8];
  load8(seed, seeds + (size_t)i * 32);
  const uint32_t o0 = off[i];
  const uint32_t len = off[i + 1] - o0;
  auto msgword = [&](uint32_t j) -> uint32_t {
    const uint32_t a = o0 + 4 * j;
    const uint32_t a0 = a & ~3u, sh = (a & 3u) * 8;
    const uint32_t lo = load_u32_guarded(msg, a0, msg_total);
    if (sh == 0) return lo;
    return __builtin_amdgcn_alignbit(load_u32_guarded(msg, a0 + 4, msg_total), lo, sh);
  };
  uint32_t pkw[8], sigw[16];
  sign_core(pkw, sigw, seed, len, msgword, tb);
  uint32_t* pko = reinterpret_cast<uint32_t*>(pk + (size_t)i * 32);
  uint32_t* sgo = reinterpret_cast<uint32_t*>(sig + (size_t)i * 64);
#pragma unroll
  for (int q = 0; q < 8; ++q) pko[q] = pkw[q];
#pragma unroll
  for (int q = 0; q < 16; ++q) sgo[q] = sigw[q];
}

// [j]B, j = 0..2^(kBWin-1), affine Niels, 32 words per entry (30 + 2 pad): built once per context
__global__ __launch_bounds__(kBlock) void build_btab_kernel(int4* __restrict__ out, int shift_words) {
  __shared__ int4 btab[AT2V_BTAB_ENTRIES * 8];
  stage_btab(btab);
  LdsTabB tb{btab};
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= (uint32_t)kBtabEntries) return;
  uint32_t sj[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int q = 0; q < 8; ++q) sj[q] = q == shift_words ? j : 0u;  // j * 2^(32 shift_words)
  ge_p2 P;
  ge_scalarmult_base(P, sj, tb);
  ge_niels nj;
  ge_p2_to_niels(nj, P);
  int32_t w[32];
#if AT2V_FIELD_FU && AT2V_VERIFY_HALF
  {  // the verify kernel reads the tables on the unsigned field
    gu_niels nu;
    niels_fe_to_fu(nu, nj);
    for (int k = 0; k < 10; ++k) {
      nj.ypx.v[k] = (int32_t)nu.ypx.v[k];
      nj.ymx.v[k] = (int32_t)nu.ymx.v[k];
      nj.xy2d.v[k] = (int32_t)nu.xy2d.v[k];
    }
  }
#endif
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    w[k] = nj.ypx.v[k];
    w[10 + k] = nj.ymx.v[k];
    w[20 + k] = nj.xy2d.v[k];
  }
  w[30] = w[31] = 0;
#pragma unroll
  for (int q = 0; q < 8; ++q) out[(size_t)j * 8 + q] = make_int4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
}

// dalek CompressedEdwardsY::decompress success bit per 32-byte point (at2v_decode_points): one lane per
// point, verdict words written per wave like the verify kernel
__global__ __launch_bounds__(kBlock) void decode_kernel(const uint8_t* __restrict__ pts, uint32_t n,
                                                        uint32_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  int ok = 0;
  if (i < n) {
    uint32_t w[8];
    load8(w, pts + (size_t)i * 32);
    ge_p3 P;
    ok = ge_frombytes(P, w);
  }
  const uint64_t mask = __ballot(ok);
  const uint32_t first = i & ~63u, nwords = (n + 31) / 32;
  if ((threadIdx.x & 63) == 0 && first < n) {
    out[first / 32] = (uint32_t)mask;
    if (first / 32 + 1 < nwords) out[first / 32 + 1] = (uint32_t)(mask >> 32);
  }
}

// ------------------------------------------------------------------ per-sender A cache kernels
// Build stream (after the launch that claimed the keys; at2v_cache.h): payloads of the claim set, then the flip that
// makes them valid. Compaction (launch stream, no cached launch or build in flight): the most recently used entries move
// to a fresh tag table, the other payloads go back to the free list.

__device__ AT2V_INLINE void entry_key(uint32_t a[8], const int4* ent) {
  const int4 k0 = ent[0], k1 = ent[1];
  a[0] = (uint32_t)k0.x; a[1] = (uint32_t)k0.y; a[2] = (uint32_t)k0.z; a[3] = (uint32_t)k0.w;
  a[4] = (uint32_t)k1.x; a[5] = (uint32_t)k1.y; a[6] = (uint32_t)k1.z; a[7] = (uint32_t)k1.w;
}

__device__ AT2V_INLINE unsigned long long claim_count(const CacheArgs& c) {
  return __hip_atomic_load(c.ctl + c.count_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Tables (combs off): one lane per claim of the set: dalek's decode verdict and [j]A (build_a_table, the verify
// kernel's own steps) into payload u; the key comes from the entry the claim wrote.
__global__ __launch_bounds__(256) void cache_build_kernel(CacheArgs c) {
  if (blockIdx.x == 0 && threadIdx.x == 0) c.ctl[kCtlBuildT0] = wall_clock64();  // (a vector store from one lane)
  const unsigned long long cnt = claim_count(c);
  for (uint32_t t = blockIdx.x * 256 + threadIdx.x; t < cnt; t += gridDim.x * 256) {
    const uint4 e = c.new_list[t];
    int4* ent = c.entries + (size_t)e.x * kCacheEntryGranules;
    uint32_t a[8];
    entry_key(a, ent);
    DevTabA tw{c.payload + (size_t)e.y * kTabAGranules, nullptr, 0, nullptr};  // store() only
    const int ok = build_a_table(a, tw);
    reinterpret_cast<int*>(ent + 2)[0] = ok;
  }
}

// One claim of the comb build: thread g of the claim's group (2^kPartsLog2 threads per position) writes its share of the
// comb of -A into payload u (comb_build_lane), g = 0 the decode verdict. The group is block- or wave-uniform.
template <int kPartsLog2>
__device__ AT2V_INLINE void comb_claim(const CacheArgs& c, uint32_t t, int g) {
  const uint4 e = c.new_list[t];
  int4* ent = c.entries + (size_t)e.x * kCacheEntryGranules;
  uint32_t a[8];
  entry_key(a, ent);
  int4* cb = c.payload + (size_t)e.y * (kCombBytes / 16);
  const int pos = g >> kPartsLog2;
  struct Mem {  // this position's entries in payload u (a lane reads back only entries it wrote itself)
    int4* row;
    __device__ AT2V_INLINE void put(int j, const uint32_t* w) const {
      int4* dst = row + (size_t)j * kCombGranules;
#pragma unroll
      for (int q = 0; q < kCombGranules; ++q)
        dst[q] = make_int4((int)w[4 * q], (int)w[4 * q + 1], (int)w[4 * q + 2], (int)w[4 * q + 3]);
    }
    __device__ AT2V_INLINE void get(int j, uint32_t* w) const {
      const int4* src = row + (size_t)j * kCombGranules;
#pragma unroll
      for (int q = 0; q < kCombGranules; ++q) {
        const int4 v = src[q];
        w[4 * q] = (uint32_t)v.x;
        w[4 * q + 1] = (uint32_t)v.y;
        w[4 * q + 2] = (uint32_t)v.z;
        w[4 * q + 3] = (uint32_t)v.w;
      }
    }
  } mem{cb + (size_t)(pos < kCombPos ? pos : 0) * kCombEntries * kCombGranules};
  const int ok = comb_build_lane<kPartsLog2>(a, pos, g & ((1 << kPartsLog2) - 1), mem);
  if (g == 0) reinterpret_cast<int*>(ent + 2)[0] = ok;
}

// Combs of a claim set (persistent grid): up to kCombWideMaxKeys claims, one 256-thread block per claim and 8 threads per
// position (profiles/r03zf); more claims, one wave per claim and 2 lanes per position (fewer redundant position chains
// once the waves outnumber the SIMDs).
__global__ __launch_bounds__(256) void cache_comb_kernel(CacheArgs c) {
  if (blockIdx.x == 0 && threadIdx.x == 0) c.ctl[kCtlBuildT0] = wall_clock64();  // (a vector store from one lane)
  const unsigned long long cnt = claim_count(c);
  if (cnt <= (unsigned long long)kCombWideMaxKeys) {
    for (uint32_t t = blockIdx.x; t < cnt; t += gridDim.x) comb_claim<kCombWideLog2>(c, t, (int)threadIdx.x);
  } else {
    const uint32_t nw = gridDim.x * 4;
    for (uint32_t t = blockIdx.x * 4 + (threadIdx.x >> 6); t < cnt; t += nw)
      comb_claim<kCombNarrowLog2>(c, t, (int)(threadIdx.x & 63));
  }
}

// After the build kernel (stream order: its payload stores are complete and written back): valid = 1 for every claim of
// the slot, then the slot's count is reset for the launch that reuses it.
__global__ __launch_bounds__(1024) void cache_flip_kernel(CacheArgs c) {
  const unsigned long long cnt = claim_count(c);
  for (uint32_t t = threadIdx.x; t < cnt; t += 1024) {
    const uint4 e = c.new_list[t];
    __hip_atomic_store(reinterpret_cast<int*>(c.entries + (size_t)e.x * kCacheEntryGranules + 2) + 1, 1,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (cnt) {  // the pass's device time (from the build kernel's first block to here) and its payload count
      c.ctl[kCtlBuildTicks] += wall_clock64() - c.ctl[kCtlBuildT0];
      c.ctl[kCtlBuilt] += cnt;
    }
    __hip_atomic_store(c.ctl + c.count_word, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// a fresh cache: every payload index free
__global__ __launch_bounds__(256) void cache_init_kernel(CacheArgs c) {
  for (uint32_t u = blockIdx.x * 256 + threadIdx.x; u < c.capacity; u += gridDim.x * 256) c.free_slots[u] = u;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    c.ctl[kCtlFreeCount] = c.capacity;
    c.ctl[kCtlFreeHead] = 0;
  }
}

__device__ AT2V_INLINE int entry_age(const CacheArgs& c, int4 m) {
  const uint32_t a = c.epoch - (uint32_t)m.w;
  return a > 63u ? 63 : (int)a;
}

// compaction 1: age histogram of the entries that hold a payload (valid: every build has been flipped by now)
__global__ __launch_bounds__(256) void cache_hist_kernel(CacheArgs c) {
  for (uint32_t s = blockIdx.x * 256 + threadIdx.x; s < c.cap; s += gridDim.x * 256) {
    if (c.tags[s] == 0) continue;
    const int4 m = c.entries[(size_t)s * kCacheEntryGranules + 2];
    if (m.y != 1 || m.z < 0) continue;
    atomicAdd(c.ctl + kCtlHist + entry_age(c, m), 1ull);
  }
}

// compaction 2 (one thread): keep every entry younger than T and `rem` of age T, at most 3/4 of the capacity, so a later
// launch has a quarter of the payloads for new keys
__global__ void cache_select_kernel(CacheArgs c) {
  const unsigned long long target = (unsigned long long)c.capacity * 3 / 4;
  unsigned long long kept = 0, rem = 0;
  int T = 64;
  for (int a = 0; a < 64; ++a) {
    const unsigned long long h = c.ctl[kCtlHist + a];
    if (kept + h > target) {
      T = a;
      rem = target - kept;
      break;
    }
    kept += h;
  }
  c.ctl[kCtlThreshold] = (unsigned long long)T;
  c.ctl[kCtlRemainder] = rem;
  c.ctl[kCtlRemTaken] = 0;
  c.ctl[kCtlKept] = 0;
  c.ctl[kCtlFreeCount] = 0;
  c.ctl[kCtlFreeHead] = 0;
  c.ctl[kCtlFull] = 0;
  c.ctl[kCtlCompactions] += 1;
}

// compaction 3: kept entries are re-inserted into the fresh tag table (their payloads stay where they are)
__global__ __launch_bounds__(256) void cache_compact_kernel(CacheArgs c, CacheCompactArgs x) {
  const int T = (int)c.ctl[kCtlThreshold];
  const unsigned long long rem = c.ctl[kCtlRemainder];
  const uint32_t mask = c.cap - 1;
  for (uint32_t s = blockIdx.x * 256 + threadIdx.x; s < c.cap; s += gridDim.x * 256) {
    const unsigned long long fp = c.tags[s];
    if (fp == 0) continue;
    const int4* e = c.entries + (size_t)s * kCacheEntryGranules;
    const int4 m = e[2];
    if (m.y != 1 || m.z < 0) continue;  // a claim that never got a payload: its tag is dropped
    const int age = entry_age(c, m);
    const bool keep = age < T || (age == T && atomicAdd(c.ctl + kCtlRemTaken, 1ull) < rem);
    if (!keep) {
      atomicAdd(c.ctl + kCtlEvicted, 1ull);
      continue;
    }
    const uint32_t h = (uint32_t)(fp >> 17) & mask;
    for (uint32_t k = 0; k < c.cap; ++k) {  // fingerprints are unique in a table: the first free tag on the path
      const uint32_t j = (h + k) & mask;
      if (atomicCAS(x.new_tags + j, 0ull, fp) == 0ull) {
        int4* d = x.new_entries + (size_t)j * kCacheEntryGranules;
        d[0] = e[0];
        d[1] = e[1];
        d[2] = m;
        x.used[m.z] = 1;
        atomicAdd(c.ctl + kCtlKept, 1ull);
        break;
      }
    }
  }
}

// compaction 4: every payload index no kept entry holds is free again
__global__ __launch_bounds__(256) void cache_freelist_kernel(CacheArgs c, CacheCompactArgs x) {
  for (uint32_t u = blockIdx.x * 256 + threadIdx.x; u < c.capacity; u += gridDim.x * 256)
    if (!x.used[u]) c.free_slots[atomicAdd(c.ctl + kCtlFreeCount, 1ull)] = u;
}

// The combs of B, D[pos][j] = [j 2^(W pos)]B for j = 0..2^(W-1), affine Niels on the unsigned field, built by additions
// (round 6, VERDICT r5 "Next" 3). Round 5 computed every entry by its own fixed-base scalar multiplication (~2,500 field
// multiplications per entry; the 20-bit table took 13 launches of ~28 ms, up to 68 ms, 68% of a profiled bench's GPU
// time). Now:
//   bcomb_base_kernel  one lane per position: P_pos = [2^(W pos)]B (W pos doublings of B, decoded from its encoding)
//                      and D_pos = [K]P_pos, both in cached form;
//   bcomb_fill_kernel  one lane per (pos, h), h < 2^(W-1)/K: S = [K h + 1]P_pos = P_pos + [h]D_pos (binary method),
//                      then its K entries j = K h + 1 .. K h + K by consecutive additions of P_pos, made affine with one
//                      inversion per lane (Montgomery's trick through the entries' own 128-byte slots, as comb_build_lane:
//                      pass 1 stores (X pi', Y pi', Z), pass 2 writes (y+x, y-x, 2dxy)); lane h = 0 also writes j = 0.
// About 30 multiplications per entry; fill launches of at most kBCombFillLanes lanes, so no launch holds the device for
// long (a node that starts beside a serving one no longer stalls it). Any representation of the same point
// gives the same verdicts; the comb paths' parity tests run on these tables.
constexpr int kBCombKLog2 = 6;
constexpr int kBCombK = 1 << kBCombKLog2;       // entries per fill lane
constexpr uint32_t kBCombFillLanes = 1u << 16;  // lanes per fill launch

__global__ __launch_bounds__(64) void bcomb_base_kernel(gu_cached* __restrict__ base, int pos_bits, int npos) {
  const int p = threadIdx.x;
  if (p >= npos) return;
  const uint32_t Bw[8] = {0x66666658u, 0x66666666u, 0x66666666u, 0x66666666u,
                          0x66666666u, 0x66666666u, 0x66666666u, 0x66666666u};  // the base point's encoding (y = 4/5)
  gu_p3 P;
  (void)gu_frombytes(P, Bw);
  gu_p2 Q2;
  gu_p1p1 t;
  const int nd = pos_bits * p;
#pragma unroll 1
  for (int d = 0; d < nd; ++d) {  // P = [2^(pos_bits p)]B
    gu_p3_to_p2(Q2, P);
    gu_p2_dbl(t, Q2);
    gu_p1p1_to_p3(P, t);
  }
  gu_cached c;
  gu_p3_to_cached(c, P);
  base[2 * p] = c;
#pragma unroll 1
  for (int d = 0; d < kBCombKLog2; ++d) {  // D = [K]P
    gu_p3_to_p2(Q2, P);
    gu_p2_dbl(t, Q2);
    gu_p1p1_to_p3(P, t);
  }
  gu_p3_to_cached(c, P);
  base[2 * p + 1] = c;
}

__device__ AT2V_INLINE void bcomb_put3(int4* dst, const fu& a, const fu& b, const fu& c) {
  uint32_t w[32];
#pragma unroll
  for (int q = 0; q < 10; ++q) {
    w[q] = a.v[q];
    w[10 + q] = b.v[q];
    w[20 + q] = c.v[q];
  }
  w[30] = w[31] = 0;
#pragma unroll
  for (int q = 0; q < 8; ++q) dst[q] = make_int4((int)w[4 * q], (int)w[4 * q + 1], (int)w[4 * q + 2], (int)w[4 * q + 3]);
}

__device__ AT2V_INLINE void bcomb_get3(const int4* src, fu& a, fu& b, fu& c) {
  uint32_t w[32];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int4 v = src[q];
    w[4 * q] = (uint32_t)v.x;
    w[4 * q + 1] = (uint32_t)v.y;
    w[4 * q + 2] = (uint32_t)v.z;
    w[4 * q + 3] = (uint32_t)v.w;
  }
#pragma unroll
  for (int q = 0; q < 10; ++q) {
    a.v[q] = w[q];
    b.v[q] = w[10 + q];
    c.v[q] = w[20 + q];
  }
}

// lanes [lane0, lane0 + grid) of the fill: lane L = pos * parts + h
__global__ __launch_bounds__(256) void bcomb_fill_kernel(int4* __restrict__ out, const gu_cached* __restrict__ base,
                                                          int bits, int npos, uint32_t lane0) {
  const uint32_t parts = (1u << (bits - 1)) >> kBCombKLog2;
  const uint32_t L = lane0 + blockIdx.x * blockDim.x + threadIdx.x;
  if (L >= parts * (uint32_t)npos) return;
  const int pos = (int)(L / parts);
  const uint32_t h = L % parts;
  const size_t entries = ((size_t)1 << (bits - 1)) + 1;
  int4* tab = out + (size_t)pos * entries * 8;
  const gu_cached P = base[2 * pos], D = base[2 * pos + 1];
  gu_p1p1 t;
  // S = [h]D + P (binary method from the top bit of h; the complete formulas take the identity)
  gu_p3 S;
  gu_p3_identity(S);
  for (int b = 31 - __builtin_clz(h | 1); b >= 0 && h; --b) {
    gu_p2 S2;
    gu_p3_to_p2(S2, S);
    gu_p2_dbl(t, S2);
    gu_p1p1_to_p3(S, t);
    if ((h >> b) & 1u) {
      gu_add(t, S, D);
      gu_p1p1_to_p3(S, t);
    }
  }
  gu_add(t, S, P);
  gu_p1p1_to_p3(S, t);
  const uint32_t j0 = h * kBCombK + 1;
  if (h == 0) {
    fu one, zero;
    fu_1(one);
    fu_0(zero);
    bcomb_put3(tab, one, one, zero);  // j = 0, the identity: y+x = 1, y-x = 1, 2dxy = 0
  }
  fu pi;  // pass 1: pi = Z_0 ... Z_m; entry m holds (X_m pi_(m-1), Y_m pi_(m-1), Z_m)
#pragma unroll 1
  for (int m = 0; m < kBCombK; ++m) {
    int4* e = tab + (size_t)(j0 + m) * 8;
    if (m == 0) {
      bcomb_put3(e, S.X, S.Y, S.Z);
      pi = S.Z;
    } else {
      fu xp, yp;
      fu_mulc(xp, S.X, pi);
      fu_mulc(yp, S.Y, pi);
      bcomb_put3(e, xp, yp, S.Z);
      fu_mulc(pi, pi, S.Z);
    }
    if (m + 1 < kBCombK) {
      gu_add(t, S, P);
      gu_p1p1_to_p3(S, t);
    }
  }
  fu inv;  // 1 / pi_m, m from the last entry down
  fu_invert(inv, pi);
#pragma unroll 1
  for (int m = kBCombK - 1; m >= 0; --m) {
    int4* e = tab + (size_t)(j0 + m) * 8;
    fu xp, yp, z, x, y;
    bcomb_get3(e, xp, yp, z);
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
    bcomb_put3(e, n.ypx, n.ymx, n.xy2d);
  }
}

size_t cache_entry_bytes() { return (size_t)kCacheEntryGranules * 16; }
size_t cache_payload_bytes(int comb) { return comb ? kCombBytes : (size_t)kTabAGranules * 16; }
size_t bcomb_bytes(int bits) {
  return bits == 24 ? BCombGeom<24>::kBytes : bits == 20 ? BCombGeom<20>::kBytes : BCombGeom<16>::kBytes;
}
int bcomb_lat_bits() { return kBCombLatBits; }
int bcomb_mid_bits() { return kBCombMidBits; }
int bcomb_wide_bits() { return kBCombBits; }

size_t bcomb_scratch_bytes() { return sizeof(gu_cached) * 2 * 16; }

// npos tables of 2^(bits-1) + 1 entries, table p = [j 2^(pos_bits p)]B: the combs of B (pos_bits = bits, every position
// of a 254-bit scalar) or the ladder's 24-bit fixed-base tables (bits 24, npos 2, pos_bits 144)
hipError_t launch_build_btables(int4* out, int bits, int npos, int pos_bits, void* scratch, hipStream_t stream) {
  if ((bits != 16 && bits != 20 && bits != 24) || npos < 1 || npos > 16) return hipErrorInvalidValue;
  gu_cached* base = static_cast<gu_cached*>(scratch);
  hipLaunchKernelGGL(bcomb_base_kernel, dim3(1), dim3(64), 0, stream, base, pos_bits, npos);
  hipError_t e = hipGetLastError();
  const uint32_t lanes = ((1u << (bits - 1)) >> kBCombKLog2) * (uint32_t)npos;
  for (uint32_t l0 = 0; l0 < lanes && e == hipSuccess; l0 += kBCombFillLanes) {
    const uint32_t k = lanes - l0 < kBCombFillLanes ? lanes - l0 : kBCombFillLanes;
    hipLaunchKernelGGL(bcomb_fill_kernel, dim3((k + 255) / 256), dim3(256), 0, stream, out, base, bits, npos, l0);
    e = hipGetLastError();
  }
  return e;
}

hipError_t launch_build_bcomb(int4* out, int bits, void* scratch, hipStream_t stream) {
  return launch_build_btables(out, bits, (254 + bits - 1) / bits, bits, scratch, stream);
}

size_t ladder_btab_bytes() { return AT2V_LADDER_BW == 24 ? (size_t)2 * kLadderEntries * 128 : 0; }
hipError_t launch_build_ladder_btab(int4* out, void* scratch, hipStream_t stream) {
  return launch_build_btables(out, 24, 2, 144, scratch, stream);
}
int cache_ctl_words() { return kCtlWords; }

static uint32_t grid_for(uint64_t items, uint32_t per_block, uint32_t cap_blocks) {
  const uint64_t b = (items + per_block - 1) / per_block;
  return (uint32_t)(b < 1 ? 1 : b > cap_blocks ? cap_blocks : b);
}

hipError_t launch_cache_init(const CacheArgs& c, hipStream_t stream) {
  hipLaunchKernelGGL(cache_init_kernel, dim3(grid_for(c.capacity, 256, 1024)), dim3(256), 0, stream, c);
  return hipGetLastError();
}

hipError_t launch_cache_build(const CacheArgs& c, uint32_t max_claims, hipStream_t stream) {
  if (max_claims == 0) max_claims = 1;
  if (c.comb) {  // a block per claim (few claims) or a wave per claim; the grid loops over more
    hipLaunchKernelGGL(cache_comb_kernel, dim3(max_claims < 512u ? max_claims : 512u), dim3(256), 0, stream, c);
    // (the kernel reads the real claim count: blocks past the keys' blocks (wide) or waves (narrow) exit at once)
  } else {
    hipLaunchKernelGGL(cache_build_kernel, dim3(grid_for(max_claims, 256, 1024)), dim3(256), 0, stream, c);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(cache_flip_kernel, dim3(1), dim3(1024), 0, stream, c);
  return hipGetLastError();
}

hipError_t launch_cache_compact(const CacheArgs& c, const CacheCompactArgs& x, hipStream_t stream) {
  hipError_t e = hipMemsetAsync(x.new_tags, 0, (size_t)c.cap * 8, stream);
  if (e == hipSuccess) e = hipMemsetAsync(x.new_entries, 0, (size_t)c.cap * kCacheEntryGranules * 16, stream);
  if (e == hipSuccess) e = hipMemsetAsync(x.used, 0, (size_t)c.capacity * 4, stream);
  if (e == hipSuccess) e = hipMemsetAsync(c.ctl + kCtlHist, 0, 64 * 8, stream);
  if (e != hipSuccess) return e;
  const uint32_t gs = grid_for(c.cap, 256, 2048), gu = grid_for(c.capacity, 256, 2048);
  hipLaunchKernelGGL(cache_hist_kernel, dim3(gs), dim3(256), 0, stream, c);
  hipLaunchKernelGGL(cache_select_kernel, dim3(1), dim3(1), 0, stream, c);
  hipLaunchKernelGGL(cache_compact_kernel, dim3(gs), dim3(256), 0, stream, c, x);
  hipLaunchKernelGGL(cache_freelist_kernel, dim3(gu), dim3(256), 0, stream, c, x);
  return hipGetLastError();
}

// ------------------------------------------------------------------ launchers (host side)

// the B tables, then (kIdentShared) the shared identity entry in cached form: YpX = 1, YmX = 1, Z2 = 2, T2d = 0
size_t btab_bytes() { return (size_t)kNumBtabs * kBtabEntries * 8 * 16 + 160; }

// table t (t = 0: [j]B; t = 1: [j 2^128]B for the half-size path) at out + t * kBtabEntries * 8
hipError_t launch_build_btab(int4* out, hipStream_t stream) {
  for (int t = 0; t < kNumBtabs; ++t) {
    hipLaunchKernelGGL(build_btab_kernel, dim3((kBtabEntries + kBlock - 1) / kBlock), dim3(kBlock), 0, stream,
                       out + (size_t)t * kBtabEntries * 8, 4 * t);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
#if AT2V_TAB_PACK  // the same entry packed (fu_pack8 of 1, 1, 2, 0)
  static const uint32_t ident[40] = {1, 0, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 0, 0, 0, 0, 2, 0, 0, 0,
                                     0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#else
  static const uint32_t ident[40] = {1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                     2, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#endif
  const hipError_t e = hipMemcpyAsync(out + (size_t)kNumBtabs * kBtabEntries * 8, ident, sizeof ident,
                                      hipMemcpyHostToDevice, stream);
  if (e != hipSuccess) return e;
  return hipStreamSynchronize(stream);  // `ident` is a host array of this function's lifetime: wait for the copy
}

size_t part_bytes_per_record() { return 12; }  // hidx, hinfo, midx

hipError_t launch_verify(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, uint32_t msg_total,
                         const uint32_t* off, uint32_t n, int policy, uint32_t* verdicts, int4* scratch,
                         const int4* btab, const int4* btab24, int grid, uint32_t pair_max, hipStream_t stream,
                         const CacheArgs* cache, const PartArgs* part, int dense, const StagedArgs* staged) {
  if (n == 0) return hipSuccess;
#if AT2V_VERIFY_HALF && AT2V_FIELD_FU
  if (n <= pair_max && !(cache && cache->comb)) {  // (with combs, small batches take the comb kernel: faster still)
    // one wave (32 records) per SIMD: 4-wave blocks; the context's scratch holds grid x 8 waves of (larger) slots
    const uint32_t nchunks = (n + 31) / 32;
    const uint32_t cap_blocks = (uint32_t)grid * kWavesPerBlock / kPairWaves;
    uint32_t g = (nchunks + kPairWaves - 1) / kPairWaves;
    g = g < cap_blocks ? g : cap_blocks;
    hipLaunchKernelGGL(verify_pair_kernel, dim3(g), dim3(kPairBlock), 0, stream, pk, sig, msg, msg_total, off, n,
                       policy, verdicts, scratch, btab);
    return hipGetLastError();
  }
#endif
  const uint32_t nchunks = (n + 63) / 64;
  // Blocks: a launch below the full grid spreads its chunks over twice as many blocks, half filled (one wave per SIMD:
  // the lowest latency for a lone batch); `dense` (the host-buffer pipeline's chunk launches, at2v_api.hip HostPipe)
  // fills every block, so a small launch takes few whole CUs at full rate and leaves the rest to the launch beside it
  // (1M records as 16 launches of 65,536: 13.3 ms half filled, one stream; profiles/r06/r06i)
  const uint32_t per_block = dense ? kWavesPerBlock : kWavesPerBlock / 2;
  const uint32_t need_blocks = (nchunks + per_block - 1) / per_block;
  const int g = (int)((uint32_t)grid < need_blocks ? (uint32_t)grid : need_blocks);
  // chunk queue counter: the word after the `grid` blocks' lane slots (scratch_bytes(grid)); the four-wave comb kernel of
  // small batches strides over its chunks and needs none (one dependent memset less on the latency path)
  uint32_t* queue = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(scratch) + (size_t)grid * kScratchPerWave * kWavesAlloc);
  const bool lat_comb = cache && cache->comb && n <= pair_max;
  const bool parted = cache && part && n > pair_max;  // (zeroes its control words itself, below)
  if (!lat_comb && !parted) {
    const hipError_t me = hipMemsetAsync(queue, 0, sizeof(uint32_t), stream);
    if (me != hipSuccess) return me;
  }
#if AT2V_VERIFY_HALF && AT2V_FIELD_FU
  if (staged) {  // the whole persistent grid: the records arrive while it runs
    if (cache) return hipErrorInvalidValue;
    hipLaunchKernelGGL(verify_kernel_staged, dim3(grid), dim3(kBlock), 0, stream, pk, n, policy, verdicts, scratch,
                       btab, btab24, queue, *staged);
    return hipGetLastError();
  }
#else
  if (staged) return hipErrorInvalidValue;
#endif
#if AT2V_VERIFY_HALF && AT2V_FIELD_FU
  if (cache && part && n > pair_max) {
    // partitioned (at2v_cache.h PartArgs): classify -> (combs) hit list by comb additions -> ladder over the rest. The
    // control words after the lane slots: [0] the ladder's chunk queue, [1] the comb kernel's, [4..5] the list sizes.
    PartArgs pa = *part;
    pa.counts = queue + 4;
    hipError_t e = hipMemsetAsync(queue, 0, 8 * sizeof(uint32_t), stream);
    if (e != hipSuccess) return e;
    const uint32_t groups = (n + 63) / 64, per_block = kClassifyWaves * kClassifyGroups;
    hipLaunchKernelGGL(cache_classify_kernel, dim3((groups + per_block - 1) / per_block), dim3(64 * kClassifyWaves), 0,
                       stream, pk, n, *cache, pa);
    if (cache->comb) {
      const uint32_t need2 = ((n + 255) / 256 + kWavesPerBlock / 2 - 1) / (kWavesPerBlock / 2);
      const int g2 = (int)((uint32_t)grid < need2 ? (uint32_t)grid : need2);
#if AT2V_EXP_COMB3
      const uint32_t need3 = ((n + 255) / 256 + 11) / 12;
      hipLaunchKernelGGL(verify_kernel_comb_part3, dim3((uint32_t)grid < need3 ? grid : need3), dim3(768), 0, stream, pk,
                         sig, msg, msg_total, off, n, policy, verdicts, scratch, queue + 1, *cache, pa);
      (void)g2;
#else
      hipLaunchKernelGGL(verify_kernel_comb_part, dim3(g2), dim3(kBlock), 0, stream, pk, sig, msg, msg_total, off, n,
                         policy, verdicts, scratch, btab, queue + 1, *cache, pa);
#endif
      hipLaunchKernelGGL(verify_kernel_miss, dim3(g), dim3(kBlock), 0, stream, pk, sig, msg, msg_total, off, n, policy,
                         verdicts, scratch, btab, btab24, queue, pa);
    } else {
      hipLaunchKernelGGL(verify_kernel_tables_part, dim3(g), dim3(kBlock), 0, stream, pk, sig, msg, msg_total, off, n,
                         policy, verdicts, scratch, btab, btab24, queue, *cache, pa);
    }
    return hipGetLastError();
  }
  if (cache) {  // the kernels look their senders up themselves (at2v_cache.h); builds follow on the build stream
    if (cache->comb && n <= pair_max) {  // small batches: the four-wave split, one block per 64 records
      const uint32_t gl = nchunks < (uint32_t)grid ? nchunks : (uint32_t)grid;
      hipLaunchKernelGGL(verify_comb_lat_kernel, dim3(gl), dim3(kLatBlock), 0, stream, pk, sig, msg, msg_total, off, n,
                         policy, verdicts, scratch, btab, *cache);
      return hipGetLastError();
    }
    if (cache->comb) {
#if AT2V_COMB_PAIRS
      const uint32_t crec = AT2V_COMB_PAIRS == 2 ? 256u : 128u;  // records per chunk
      const uint32_t need2 = ((n + crec - 1) / crec + kWavesPerBlock / 2 - 1) / (kWavesPerBlock / 2);
      const int g2 = (int)((uint32_t)grid < need2 ? (uint32_t)grid : need2);
#else
      const int g2 = g;
#endif
      hipLaunchKernelGGL(verify_kernel_comb, dim3(g2), dim3(kBlock), 0, stream, pk, sig, msg, msg_total, off, n, policy,
                         verdicts, scratch, btab, queue, *cache);
      return hipGetLastError();
    }
    hipLaunchKernelGGL(verify_kernel_cached, dim3(g), dim3(kBlock), 0, stream, pk, sig, msg, msg_total, off, n, policy,
                       verdicts, scratch, btab, btab24, queue, *cache);
    return hipGetLastError();
  }
#endif
  hipLaunchKernelGGL(verify_kernel, dim3(g), dim3(kBlock), 0, stream, pk, sig, msg, msg_total, off, n, policy,
                     verdicts, scratch, btab, btab24, queue);
  return hipGetLastError();
}

hipError_t launch_gen(uint64_t cfg, uint64_t first, uint32_t n, uint32_t msg_len, uint64_t senders,
                      const uint64_t* keys, uint8_t* pk, uint8_t* sig, uint8_t* msg, uint32_t* off, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(gen_kernel, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, stream, cfg, first, n, msg_len,
                     senders, keys, pk, sig, msg, off);
  return hipGetLastError();
}

hipError_t launch_sign(const uint8_t* seeds, const uint8_t* msg, uint32_t msg_total, const uint32_t* off, uint32_t n,
                       uint8_t* pk, uint8_t* sig, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(sign_kernel, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, stream, seeds, msg, msg_total, off,
                     n, pk, sig);
  return hipGetLastError();
}

hipError_t launch_decode(const uint8_t* pts, uint32_t n, uint32_t* out, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(decode_kernel, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, stream, pts, n, out);
  return hipGetLastError();
}

hipError_t verify_occupancy(int* blocks_per_cu, int* vgprs) {
  hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, verify_kernel, kBlock, 0);
  if (e != hipSuccess) return e;
  hipFuncAttributes attr;
  e = hipFuncGetAttributes(&attr, reinterpret_cast<const void*>(verify_kernel));
  if (e == hipSuccess && vgprs) *vgprs = attr.numRegs;
  return e;
}

size_t scratch_bytes_per_block() { return kScratchPerWave * kWavesAlloc; }
// device scratch of a context launching `grid` blocks: their lane slots + the chunk queue counter
size_t scratch_bytes(int grid) { return (size_t)grid * scratch_bytes_per_block() + kCtlBytes(grid); }
int block_threads() { return kBlock; }

// The timing-only experiment switches compiled into this object (each gives WRONG verdicts): a bitmask of
// AT2V_EXPERIMENT_* (include/at2v.h). at2v_create refuses such a build unless AT2V_ALLOW_EXPERIMENT=1.
unsigned kernel_experiments() {
  unsigned m = 0;
#if AT2V_EXP_TAB128
  m |= AT2V_EXPERIMENT_TAB128;
#endif
#if AT2V_EXP_COMB_HOT
  m |= AT2V_EXPERIMENT_COMB_HOT;
#endif
#if AT2V_EXP_SLOT_WAVES
  m |= AT2V_EXPERIMENT_SLOT_WAVES;
#endif
#if AT2V_EXP_CONST_MSG
  m |= AT2V_EXPERIMENT_CONST_MSG;
#endif
#if AT2V_EXP_COMB3
  m |= AT2V_EXPERIMENT_COMB3;
#endif
  return m;
}

}  // namespace at2v

#ifdef AT2V_COMB_PROBE
// probe builds only: copy out the comb kernel's probe sums (at2v::kCpN counters) and zero them
extern "C" int at2v_probe_read(unsigned long long* out, int n) {
  if (n < (int)at2v::kCpN) return -1;
  if (hipDeviceSynchronize() != hipSuccess) return -2;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(at2v::at2v_cprobe_acc), sizeof(unsigned long long) * at2v::kCpN) !=
      hipSuccess)
    return -3;
  unsigned long long z[at2v::kCpN] = {};
  if (hipMemcpyToSymbol(HIP_SYMBOL(at2v::at2v_cprobe_acc), z, sizeof(z)) != hipSuccess) return -4;
  return (int)at2v::kCpN;
}
#endif
