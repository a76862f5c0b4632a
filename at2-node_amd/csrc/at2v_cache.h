// at2v_cache.h — device buffers of the per-sender A cache (at2v_opts.sender_cache), shared by the launcher
// (at2v_kernels.hip) and the context (at2v_api.hip). AT2 senders issue consecutive sequences
// (/root/reference/src/bin/server/accounts/account.rs:36-43), so one key signs many payloads of a node batch; the cache
// keeps, per distinct A, dalek's decode verdict and a payload derived from A alone: the table [j]A the ladder kernel
// would otherwise rebuild per record, or (sender_comb) the comb of -A that replaces the doublings.
//
// Layout (round 4):
//   tags[cap]      64-bit keyed fingerprints, 0 = free (open addressing, cap >= 2 x capacity: load <= 1/2)
//   entries[cap]   4 granules: key (A's 32 bytes), meta = {decode verdict, valid, payload index u (-1: none), last epoch}
//   payload[u]     capacity payloads (a table [j]A or a comb), handed out from the free list free_slots[]
// The verify kernels look their senders up themselves (chunk prologue) and claim new keys; a claim takes a payload
// index from the free list and is listed in the launch's claim slot. After the launch the context's build stream builds
// the payloads (cache_build_kernel / cache_comb_kernel), then cache_flip_kernel sets valid and frees the slot: a key
// becomes usable by launches that start later, and the launch that first sees it verifies its records without the cache,
// never waiting for a build.
// When the free list runs dry the launch flags the cache full; the context then compacts it on the build stream (round
// 5: asynchronously; launches issued meanwhile read the old table and claim nothing): the most recently used entries (by
// launch epoch, at most 3/4 of the capacity) move to the spare tag table with their payloads in place, every other
// payload goes back to the free list, and a later launch swaps the tables once the compaction has completed. A key
// claims a payload only at its second sighting (admission, CacheArgs::seen).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace at2v {

struct CacheArgs {
  unsigned long long* tags;  // cap fingerprints (cap a power of two)
  uint32_t cap;
  uint32_t capacity;         // payload slots
  int4* entries;             // cap x kCacheEntryGranules (zeroed at creation / compaction: every entry invalid)
  int4* payload;             // capacity x cache_payload_granules()
  uint32_t* free_slots;      // payload indices; [free_head, free_count) are free (ctl words)
  uint4* new_list;           // a claim list: (entry slot, payload u, 0, 0) per claim that got a payload
  int count_word;            // the list's count (ctl word kCtlClaims0 + claim slot)
  uint32_t epoch;            // launch number (entries record the last one that used them)
  int comb;                  // 1: payloads are combs of -A (sender_comb), 0: tables [j]A
  const int4* bcomb_lat;     // sender_comb: the comb of B, 16-bit windows (kBCombLatBits; 67 MB, MALL-resident)
  const int4* bcomb;         // sender_comb: the hit-list kernel's comb of B: kBCombMidBits-bit windows (872 MB), or
                             // with AT2V_CTX_BCOMB_WIDE kBCombBits-bit ones (11.8 GB)
  int bcomb_bits;            // bcomb's window (20 or 24)
  unsigned long long* ctl;   // counters, kCtl* in at2v_kernels.hip
  uint64_t seed;             // fingerprint key (random per context)
  uint64_t fp_mask;          // fingerprint bits kept (all in the product; fewer in a test that forces collisions)
  // Admission (round 5): a key not in the table claims a tag and a payload only if it was sighted before (its
  // fingerprint is in the direct-mapped sighting filter seen[], written by an earlier unadmitted sighting, in this launch
  // or an earlier one), if two or more records of the wave carry it, or with admit_first. Otherwise the leader lane
  // writes the fingerprint into seen[] and the records are verified without the cache: a one-shot sender costs one
  // 8-byte store instead of a 1.7 MB comb build and a payload (VERDICT r4 "missing" 3).
  unsigned long long* seen;  // seen_mask + 1 fingerprints (0 = empty)
  uint32_t seen_mask;
  int admit_first;           // AT2V_CTX_ADMIT_FIRST: every new key claims at once (round-4 behaviour)
  int no_claim;              // this launch only looks keys up (a compaction of the tag table is running on the build
                             // stream: the launch reads the old table, claims nothing, so the free list stays intact)
};

// Partitioned cached launch (round 5, launches above small_batch_max): cache_classify_kernel looks every record's sender
// up (claims, sightings, statistics) and splits the launch's record indices into a hit list (with each hit's payload
// index and decode verdict) and a miss list; the comb kernel then verifies the hit list by comb additions, four records
// per lane, and the ladder kernel the miss list (with [j]A tables: the hit list too, skipping A's decode). So a record
// takes the cached path whenever ITS sender is cached, whatever the other records of its chunk; round 4 required all
// 256 records of a chunk to hit, which mixed traffic (many senders) almost never does.
struct PartArgs {
  uint32_t* hidx;    // record indices of the hits (counts[0] of them, in no particular order)
  uint32_t* hinfo;   // per hit: (payload index << 1) | dalek decode verdict of A
  uint32_t* midx;    // record indices of the misses (counts[1])
  uint32_t* counts;  // [0] hits, [1] misses (zeroed before the classify kernel)
};
size_t part_bytes_per_record();

// A host-buffer batch verified by ONE launch while its records are still being uploaded (at2v_api.hip, the staged
// form of the host pipeline). The shard's records are in nreg regions of 2^ushift records (the last one: last_c), each
// laid out as chunk_layout (pk | sig | rebased offsets | messages, mb[u] bytes) at at[u] of the device arena. The host
// publishes how many regions have landed in a pinned word, (epoch << 32) | count (bit 31 of count: abort); a wave
// entering region u polls it until count > u, then takes a system-scope acquire (HSA: the receiving device's acquire
// before using DMA-written data). No region's lines are read before it is published, and regions are 256-byte aligned,
// so no cache holds a line of it from before.
constexpr int kMaxStageRegions = 64;
struct StagedArgs {
  uint64_t at[kMaxStageRegions];  // region offsets in the launch's arena argument (pointers derived from a restrict
                                  // kernel argument keep its no-alias guarantee)
  uint32_t mb[kMaxStageRegions];
  const unsigned long long* ready;  // pinned host word
  uint32_t* timeout;                // pinned host word: a wave gave up waiting (kStageTimeoutTicks)
  uint32_t epoch, ushift, nreg, last_c;
  uint32_t nap;  // s_sleep(8) rounds between two polls
};

// compaction work buffers (one per device; the alternate tag/entry arrays are swapped in by the host)
struct CacheCompactArgs {
  unsigned long long* new_tags;
  int4* new_entries;
  uint32_t* used;  // capacity flags: payload kept
};

size_t cache_entry_bytes();
size_t cache_payload_bytes(int comb);  // one key's payload: table [j]A or comb
size_t bcomb_bytes(int bits);          // a comb of B with bits-bit windows (16, 20 or 24)
int bcomb_lat_bits();
int bcomb_mid_bits();
int bcomb_wide_bits();
// build a comb of B into out (bcomb_bytes(bits)), asynchronously on stream; scratch: bcomb_scratch_bytes() of device
// memory the launches use until they complete
size_t bcomb_scratch_bytes();
hipError_t launch_build_bcomb(int4* out, int bits, void* scratch, hipStream_t stream);
int cache_ctl_words();
// ctl word indices the host reads (at2v_get_info) and resets
enum CacheCtlWord : int {
  kCtlFreeHead = 0,  // payload indices handed out since the last compaction
  kCtlFreeCount,     // free payload indices after the last compaction
  kCtlFull,          // a claim found the free list empty (or a probe path full): compact before the next launch
  kCtlClaims0,       // claims (with a payload) listed in claim slots 0..7, reset by the slot's flip kernel
  kCtlClaims7 = kCtlClaims0 + 7,
  kCtlFound,         // records whose key had a tag (statistics)
  kCtlClaimed,       // keys claimed
  kCtlFailed,        // records that found neither their key nor a free tag on the probe path
  kCtlChunkHits,     // chunks whose records all had a valid entry
  kCtlChunks,
  kCtlEvicted,       // entries dropped by compactions (total)
  kCtlCompactions,
  kCtlKept,          // scratch words of a compaction
  kCtlThreshold,
  kCtlRemainder,
  kCtlRemTaken,
  kCtlSighted,       // first sightings recorded in seen[] instead of a claim (admission)
  kCtlBuildT0,       // device wall clock (wall_clock64) when the current build pass started
  kCtlBuildTicks,    // wall-clock ticks of every build pass that built something (at2v_info.cache_build_us)
  kCtlBuilt,         // payloads built
  kCtlRecHits,       // records whose sender was served from the cache (partitioned launches)
  kCtlHist,          // 64 age buckets
  kCtlWordsTotal = kCtlHist + 64
};
// initialise a fresh cache: free list 0..capacity-1 (stream order)
hipError_t launch_cache_init(const CacheArgs& c, hipStream_t stream);
// build stream, after the launch that filled claim slot c (c.new_list, count word c.count_word): build the payloads it
// claimed, mark them valid, reset the slot's count
hipError_t launch_cache_build(const CacheArgs& c, uint32_t max_claims, hipStream_t stream);
// compact a full cache into (x.new_tags, x.new_entries) (stream order; no cached launch or build may be in flight)
hipError_t launch_cache_compact(const CacheArgs& c, const CacheCompactArgs& x, hipStream_t stream);

}  // namespace at2v
