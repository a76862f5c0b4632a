// at2v_cache.h — device buffers of the per-sender A cache (at2v_opts.sender_cache), shared by the launcher
// (at2v_kernels.hip) and the context (at2v_api.hip). AT2 senders issue consecutive sequences
// (/root/reference/src/bin/server/accounts/account.rs:36-43), so one key signs many payloads of a node batch; the cache
// keeps, per distinct A, dalek's decode verdict and the table [j]A the verify kernel would otherwise rebuild per record.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace at2v {

struct CacheArgs {
  unsigned long long* tags;  // cap 64-bit fingerprints, 0 = free (cap a power of two)
  uint32_t cap;
  uint32_t capacity;         // entries built since the last restart (<= cap / 2); claims beyond it stay unbuilt
  int4* entries;             // cap entries of cache_entry_granules() x 16 B (zeroed at creation: every entry invalid)
  int* slot_of;              // per record of the launch: entry index or -1
  uint4* new_list;           // (entry, record, claim index since the restart, 0) of the entries claimed by this launch
  int4* comb;                // at2v_opts.sender_comb: capacity combs of kCombBytes (claim index u -> comb u), else null
  const int4* bcomb;         // ... and the context's comb of B (kBCombPos x kBCombEntries affine Niels entries)
  unsigned long long* ctl;   // counters, kCtl* in at2v_kernels.hip: used, full, new, found, claimed, failed, chunk hits
  uint64_t seed;             // fingerprint key (random per context)
  uint64_t fp_mask;          // fingerprint bits kept (all in the product; fewer in a test that forces collisions)
};

size_t cache_entry_bytes();
size_t comb_bytes();   // one key's comb
size_t bcomb_bytes();  // the comb of B
hipError_t launch_build_bcomb(int4* out, hipStream_t stream);
int cache_ctl_words();
// ctl word indices the host reads (at2v_get_info) and resets
int cache_ctl_used();
int cache_ctl_full();
int cache_ctl_chunk_hits();
int cache_ctl_chunks();
// lookup / claim the launch's senders, then build the entries it claimed (stream order: before the verify kernel)
hipError_t launch_cache_prepare(const CacheArgs& c, const uint8_t* pk, uint32_t n, hipStream_t stream);

}  // namespace at2v
