// at2v_api.hip — the C ABI of include/at2v.h (host side).
//
// A context owns, per device: a stream, the persistent-grid scratch for the per-lane A tables,
// and growable device staging buffers for host batches. Host batches are split by index range
// (aligned to 64 records = one wave chunk = two verdict words) across the context's devices;
// each shard runs H2D -> verify -> D2H on its own stream, so shards overlap.
//
// Every verify launch of a context goes through launch_shard(). A device has kScratchSets scratch sets (per-wave tables,
// chunk-queue counter, pacing lines) used in turn: a launch waits only for the launch that last used its set (an event,
// whatever stream that ran on), so launches on DIFFERENT caller streams overlap: the next batch's blocks take the CUs the
// previous launch's last blocks leave, instead of the device idling through its end-of-launch drain (+3.6% on
// back-to-back config-2 batches, profiles/r03i). The verdict words are zeroed before the kernel, so a chunk that no wave
// wrote fails closed.
//
// Multi-process (one rank per GPU): at2v_comm_init_rank attaches an RCCL communicator to a
// context; at2v_verify_shard_gather_device / at2v_verify_batch_sharded verify this rank's index range and
// ncclAllGather the verdict words over xGMI, so every rank holds the node bitmap (rpc.rs:156-173 consumer).
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/at2v.h"
#include "at2v_cache.h"
#include "at2v_cpu.h"
#include "at2v_env.h"
#include "at2v_shard.h"

namespace at2v {
hipError_t launch_verify(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, uint32_t msg_total,
                         const uint32_t* off, uint32_t n, int policy, uint32_t* verdicts, int4* scratch,
                         const int4* btab, const int4* btab24, int grid, uint32_t pair_max, hipStream_t stream,
                         const CacheArgs* cache, const PartArgs* part, int dense, const StagedArgs* staged);
size_t btab_bytes();
size_t ladder_btab_bytes();
hipError_t launch_build_ladder_btab(int4* out, void* scratch, hipStream_t stream);
hipError_t launch_build_btab(int4* out, hipStream_t stream);
hipError_t launch_gen(uint64_t cfg, uint64_t first, uint32_t n, uint32_t msg_len, uint64_t senders,
                      const uint64_t* keys, uint8_t* pk, uint8_t* sig, uint8_t* msg, uint32_t* off, hipStream_t stream);
hipError_t launch_sign(const uint8_t* seeds, const uint8_t* msg, uint32_t msg_total, const uint32_t* off, uint32_t n,
                       uint8_t* pk, uint8_t* sig, hipStream_t stream);
hipError_t launch_decode(const uint8_t* pts, uint32_t n, uint32_t* out, hipStream_t stream);
hipError_t verify_occupancy(int* blocks_per_cu, int* vgprs);
size_t scratch_bytes_per_block();
size_t scratch_bytes(int grid);
int block_threads();
unsigned kernel_experiments();
}  // namespace at2v

namespace {

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    const size_t want = std::max<size_t>(bytes + bytes / 4, 4096);
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

// Per-sender A cache of one device (at2v_opts.sender_cache; at2v_cache.h). Cached launch L claims new keys
// into claim slot b = L % kClaimSlots; after the launch the build stream (the context's own stream) builds the slot's
// payloads, flips them valid, frees the slot (slot_free[b]) and copies the counters for the host, so no launch waits for
// a build unless kClaimSlots launches in a row are still waiting for theirs. When a launch finds the free list empty,
// the host learns it from that copy and enqueues a compaction on the build stream (cache_before_launch); no launch waits
// for it.
constexpr int kClaimSlots = 8;
struct PendingBuild {  // a launch's builds, enqueued on the build stream after it
  at2v::CacheArgs args{};
  uint32_t max_claims = 0;
  int slot = 0;
};
struct SenderCache {
  at2v::CacheArgs args{};
  DevBuf tags[2], entries[2];  // the live tag table / entries ([cur]) and the compaction target ([cur ^ 1])
  int cur = 0;
  DevBuf payload, free_slots, used, ctl, seen, claim_list[kClaimSlots];
  const int4* bcomb = nullptr;      // the combs of B, shared by the process's comb contexts on this device (bcomb_acquire)
  const int4* bcomb_lat = nullptr;
  // Builds run on the context's own stream (the shard's), which a caller's launches on its own streams never use: a
  // separate build stream would share one of the process's 4 hardware queues (GPU_MAX_HW_QUEUES, round robin) with a
  // caller's stream, whose next copy or launch then waited behind a 0.8 ms comb build (config 5 p99).
  hipStream_t build = nullptr;
  hipEvent_t claims_ready[kClaimSlots] = {};  // launch stream, after the launch that filled slot b
  hipEvent_t slot_free[kClaimSlots] = {};     // build stream, after slot b's flip
  hipEvent_t built = nullptr;                 // build stream, after the last flip
  // recorded after the last compaction (build stream). Until it has completed, launches read the old table and claim
  // nothing; the first launch after it swaps the tables. So no launch probes a tag table that is still being filled or
  // pops the free list while it is being rebuilt, whatever stream it runs on (in round 4 a launch on the other
  // scratch set's stream could overlap a compaction enqueued on its neighbour's stream).
  hipEvent_t compacted = nullptr;
  unsigned long long* host_ctl = nullptr;  // pinned copy of the device counters, refreshed after every cached launch
  hipEvent_t ctl_copied = nullptr;
  bool copy_pending = false;
  bool compact_pending = false;  // a launch found the cache full: compact before a later launch
  bool compacting = false;       // a compaction is enqueued on the build stream and has not been swapped in yet
  uint64_t launches = 0;  // launch epochs (entries record the last launch that used them)
  // Thrash guard (round 6, VERDICT r5 "Next" 2): a compaction that had to evict entries used by the latest launch
  // (its age threshold is 0: the working set is larger than the cache and every cached key is still in use) would only
  // trade comb builds for other keys of the same worth. The cache then stops claiming for freeze_len launches (8,
  // doubling up to 256 while compactions keep cutting at age 0; a compaction that cuts older entries resets it), so the
  // keys it holds keep serving and no build is spent on churn.
  uint64_t compactions_seen = 0;
  uint32_t freeze_len = 0, freeze_left = 0;
};

// scratch sets per device (AT2V_SCRATCH_SETS overrides, 1..4; 1 = every launch waits for the previous one)
constexpr int kScratchSets = 2;

// The host-buffer path (at2v_verify_batch, at2v_verify_batch_sharded; round 6, VERDICT r5 "Next" 1). A shard's records go
// to the device in chunks through kStageSlots pinned staging buffers, so the three stages of consecutive chunks overlap:
//   host     the copy pool's threads copy chunk i from the caller's (pageable) arrays into slot i % kStageSlots, packed
//            as pk | sig | rebased offsets | messages;
//   copy     DMA uploads on the shard's copy stream into the chunk's own region of the pipe's device arena;
//   compute  the verify launch of chunk i on compute stream i % 2 (two streams on two hardware queues: launch i+1 takes
//            the CUs launch i leaves during its end-of-launch drain), writing the chunk's verdict words of the shard's
//            device bitmap; dense grids (whole CUs per block), so small chunks run at full rate beside each other.
// The host refills a pinned slot once its upload is done (`uploaded`, host wait). The first two chunks are half a device
// each (the pipeline's fill: nothing runs until the first is up), later ones kStageMaxRecords, one full round of the
// persistent grid. Splitting a batch into such launches costs nothing on the device (1M records as 8 launches of 131,072:
// 9.30 ms on two streams against 9.34 ms for one launch, profiles/r06/r06j). Round 1 measured the previous form of this call
// (pageable hipMemcpyAsync, then verify, then D2H) at 54 M/s against a 78 M/s kernel; the stages were serial.
constexpr int kStageSlots = 3;
constexpr size_t kStageMaxRecords = 131072;  // 2,048 wave chunks: one per resident wave of the persistent grid
constexpr size_t kStageFirstRecords = 65536;  // 1,024 wave chunks: half the device in dense blocks
constexpr size_t kCopyPiece = 1 << 20;       // bytes per copy-pool job item
constexpr size_t kCopyPoolMin = 2 << 20;     // chunks below this many bytes are copied by the calling thread alone
constexpr size_t kCopyBatch = 8;             // copy pieces between two polls of the pending chunk's uploads
struct ChunkLaunch {  // a staged chunk's launch: where its parts are on the device, where its verdict words go
  uint8_t* d = nullptr;
  size_t sig = 0, off = 0, msg = 0, mb = 0, c = 0;
  uint32_t* d_words = nullptr;
  bool throughput = false;
  int slot = 0, stream = 0;
};
struct StageSlot {
  uint8_t* host = nullptr;  // pinned
  size_t host_cap = 0;
  hsa_signal_t uploaded{0};  // the slot's DMA uploads: set to their count, each decrements it as it completes
};
// The staged form (test hook AT2V_TEST_STAGED=1, a context without a sender cache, a shard part above small_batch_max):
// ONE launch of the persistent grid over the shard's whole part, issued before any record is uploaded; the records go up
// in regions of 2^ushift records (>= 65,536, at most kMaxStageRegions) through the same slots and DMA uploads, and the
// host publishes each landed region in a pinned word the waves poll (at2v_cache.h StagedArgs). Correct (the parity tests
// run it), but slower than the chunk launches: 12.4-14.9 ms per 1M records against 11.0-11.7 (profiles/r06/r06o-r06v). The
// device's clock follows its activity: a launch after 1 ms idle takes 10.5 ms instead of 9.6 (6 ms idle: 11.0, profiles/r06/r06u),
// and a grid whose waves sleep while they wait for regions looks idle; chunk launches start only when their records are
// up. Kept behind the hook for that measurement.
struct StagedCtl {
  unsigned long long ready;  // (epoch << 32) | regions published; bit 31 of the count: abort
  uint32_t timeout;          // set by a wave that gave up waiting
};
struct StagedPlan {  // one shard's part of a host-buffer call in the staged form
  bool active = false;
  size_t m = 0, lo = 0;  // records, first record (absolute)
  uint32_t ushift = 16, nreg = 0, submitted = 0, published = 0;
  std::vector<size_t> at;  // region offsets in the pipe's arena
  int slot_region[3] = {-1, -1, -1};
  at2v::StagedArgs args{};
  uint32_t* verdicts = nullptr;  // the call's device bitmap for this shard
  bool launched = false;
};
constexpr size_t kStageRegionMinLog2 = 16;

struct HostPipe {
  hipStream_t copy = nullptr;                 // the verdict download, (sharded) the all-gathers
  hipStream_t comp[2] = {nullptr, nullptr};   // verify launches of the chunks, alternating
  hipEvent_t comp_done[2] = {nullptr, nullptr};
  StageSlot slot[kStageSlots];
  DevBuf arenas[3];     // a call's chunks on the device, each in its own region (arena_at: the next free byte); one
  int cur = 0;          // arena per host-buffer call slot (HostCall slot `cur`, allocated when first used)
  size_t arena_at = 0;
  DevBuf& arena() { return arenas[cur]; }
  hsa_agent_t gpu{0}, cpu{0};  // the DMA uploads' destination and source agents
  bool pending = false;  // a chunk whose uploads are submitted and whose launch is not issued yet
  ChunkLaunch pend;
  uint64_t chunks = 0;  // chunks issued by this shard (slot chunks % kStageSlots, compute stream chunks % 2)
  StagedCtl* ctl = nullptr;  // pinned, fine-grained (the staged form)
  uint32_t epoch = 0;
};

struct Shard {
  int device = 0;
  hipStream_t stream = nullptr;
  int sets = kScratchSets;
  unsigned next_set = 0;
  hipEvent_t scratch_free[4] = {};  // per set: recorded after the launch that last used it; the set's next launch waits
  int grid = 0;  // persistent grid (blocks)
  int cus = 0;
  int blocks_per_cu = 0;
  int vgprs = 0;
  DevBuf scratch[4];
  DevBuf part[4];  // per scratch set: the classify kernel's hit / miss lists (partitioned cached launches)
  DevBuf btab, pk, sig, msg, off, verdict;
  const int4* btab24 = nullptr;  // the throughput ladder's 24-bit fixed-base tables, shared per device (bcomb_acquire)
  hipEvent_t copied = nullptr;  // the verdict copy of a device-side call (decode, sharded)
  DevBuf hverdict[3];            // host-buffer calls: the shard's device bitmap per call slot (HostCall)
  hipEvent_t hcopied[3] = {nullptr, nullptr, nullptr};  // ... and its verdict copy (the call waits for this, not for
                                                        // the cache builds behind it)
  SenderCache* cache = nullptr;
  HostPipe* pipe = nullptr;     // the host-buffer path's streams and staging (created by the first host-buffer call)
};

}  // namespace

// A host-buffer call in flight. Slots 0 and 1: at2v_verify_batch_submit (slot = ticket % 2; at most two in flight, each
// with its own device bitmap and arena per shard, so the host stages the second while the first one's launches run and
// the device sees no gap between them). Slot 2: the synchronous at2v_verify_batch, after the calls in flight are
// complete (their results stay for their waits).
struct HostCall {
  bool active = false, done = false;
  uint64_t ticket = 0;
  int rc = 0;
  const uint8_t *pk = nullptr, *sig = nullptr, *msg = nullptr;
  const uint32_t* msg_off = nullptr;
  uint32_t* verdicts = nullptr;
  size_t n = 0;
  std::vector<hipError_t> err;  // per shard
  std::vector<size_t> m;        // per shard: records
  std::vector<char> staged;     // per shard: the staged form (its timeout word is checked)
  std::chrono::steady_clock::time_point t0;
};

// verdict words per rank per all-gather round of at2v_verify_batch_sharded (2M records per rank per round)
constexpr size_t kGatherWindow = 65536;

struct at2v_ctx {
  at2v_policy policy = AT2V_POLICY_DALEK_V1;
  uint32_t pair_max = AT2V_SMALL_BATCH_DEFAULT;  // launches of <= this many records: low-latency kernel
  uint32_t flags = 0;         // at2v_opts.flags (AT2V_CTX_*)
  std::vector<Shard> shards;  // empty: a CPU-backend context (at2v_opts.num_gpus = 0)
  at2v::CpuPool* cpu = nullptr;  // the CPU backend (a CPU context, or AT2V_CTX_CPU_FALLBACK)
  at2v::CpuPool* copier = nullptr;  // the host-buffer path's staging copies (created by the first host-buffer call)
  // atomic: an ingest queue with AT2V_QUEUE_CPU_FALLBACK may fall back from its launcher and its completer thread at once
  // (both call at2v_verify_batch on the queue's CPU context; the pool serialises the work itself)
  std::atomic<uint64_t> cpu_batches{0}, cpu_fallbacks{0};
  // the host-buffer path's chunk schedule (HostPipe; test hooks AT2V_TEST_STAGE_FIRST / _MAX / AT2V_TEST_COPY_THREADS)
  size_t stage_first = kStageFirstRecords, stage_max = kStageMaxRecords;
  unsigned copy_threads = 8;
  int pipe_streams = 0;     // create_comp_stream mode (test hook AT2V_TEST_PIPE_STREAMS)
  bool staged = false;      // test hook AT2V_TEST_STAGED=1: the staged form where it applies (not faster, see StagedCtl)
  uint32_t stage_nap = 2;   // StagedArgs.nap (test hook AT2V_TEST_STAGE_NAP)
  uint32_t stage_launch_at = 0;  // test hook AT2V_TEST_STAGE_LAUNCH_AT: the launch once this many regions are published
  bool stage_pre = false;   // test hook AT2V_TEST_STAGE_PRE: every region uploaded before the launch (kernel-only time)
  bool pipe_trace = false;  // test hook AT2V_TEST_PIPE_TRACE: per host-buffer call, where the host's time went (stderr)
  double tr_wait = 0, tr_copy = 0, tr_enq = 0;  // seconds, this call
  uint64_t host_chunks = 0;  // chunks staged by host-buffer calls (at2v_info.host_chunks)
  uint32_t test_fail_launches = 0;  // AT2V_TEST_FAIL_LAUNCH (tests only): that many launches fail before the kernel
  bool partition = true;  // cached launches above pair_max classify, then verify hits and misses apart (AT2V_CACHE_PARTITION)
  ncclComm_t comm = nullptr;  // at2v_comm_init_rank (one rank per process, the context's first device)
  int rank = 0, world = 1;
  DevBuf window;              // at2v_verify_batch_sharded: world x kGatherWindow words, one all-gather round
  DevBuf zeros;               // >= kGatherWindow zero words: what a rank that failed locally sends
  DevBuf zeros_big;           // zero words for at2v_verify_shard_gather_device calls with words_per_rank > kGatherWindow
  DevBuf status;              // one int32: the cross-rank failure flag (at2v_verify_batch_sharded)
  hipEvent_t gather_done = nullptr;  // recorded after every all-gather, on its stream (at2v_destroy waits for it)
  uint64_t gathers = 0;       // all-gathers issued (at2v_info.gathers)
  HostCall calls[3];          // host-buffer call slots (HostCall)
  uint64_t next_ticket = 1;
};

namespace {

int hip_code(hipError_t e) {
  if (e == hipSuccess) return AT2V_OK;
  if (e == hipErrorOutOfMemory) return AT2V_E_OOM;
  if (e == hipErrorNoDevice || e == hipErrorInvalidDevice || e == hipErrorNoBinaryForGpu) return AT2V_E_NODEVICE;
  return AT2V_E_HIP;
}

#define AT2V_TRY(expr)                       \
  do {                                       \
    hipError_t e_ = (expr);                  \
    if (e_ != hipSuccess) return hip_code(e_); \
  } while (0)

constexpr int kLadderKey = -24;  // bcomb_acquire's key for the ladder tables (the combs use their window width)
hipError_t bcomb_acquire(int device, int bits, hipStream_t st, const int4** out);
void bcomb_release(const int4* p);

int init_shard(Shard& s, int device) {
  s.device = device;
  AT2V_TRY(hipSetDevice(device));
  hipDeviceProp_t prop;
  AT2V_TRY(hipGetDeviceProperties(&prop, device));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return AT2V_E_NODEVICE;
  s.cus = prop.multiProcessorCount;
  AT2V_TRY(at2v::verify_occupancy(&s.blocks_per_cu, &s.vgprs));
  if (s.blocks_per_cu < 1) s.blocks_per_cu = 1;
  s.grid = s.cus * s.blocks_per_cu;
  AT2V_TRY(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
  AT2V_TRY(hipEventCreateWithFlags(&s.copied, hipEventDisableTiming));
  for (hipEvent_t& ev : s.hcopied) AT2V_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));  // (3 slots)
  if (const char* v = at2v::test_env("AT2V_SCRATCH_SETS")) s.sets = std::min(4, std::max(1, std::atoi(v)));
  for (int j = 0; j < s.sets; ++j) {
    AT2V_TRY(hipEventCreateWithFlags(&s.scratch_free[j], hipEventDisableTiming));
    AT2V_TRY(hipEventRecord(s.scratch_free[j], s.stream));
    AT2V_TRY(s.scratch[j].ensure(at2v::scratch_bytes(s.grid)));
  }
  // fixed-base table [0..2^(AT2V_BWIN-1)]B, built on the device once per context
  AT2V_TRY(s.btab.ensure(at2v::btab_bytes()));
  AT2V_TRY(at2v::launch_build_btab((int4*)s.btab.p, s.stream));
  AT2V_TRY(hipStreamSynchronize(s.stream));
  // the throughput kernels' 24-bit tables [j]B, [j 2^144]B (2 GB, kernels' AT2V_LADDER_BW), one copy per device
  if (at2v::ladder_btab_bytes()) AT2V_TRY(bcomb_acquire(device, kLadderKey, s.stream, &s.btab24));
  return AT2V_OK;
}

bool aligned(const void* p, size_t a) { return (reinterpret_cast<uintptr_t>(p) & (a - 1)) == 0; }

// The combs of B, shared by every comb context of the process on a device (round 6, VERDICT r5 "Next" 3): built by the
// first context that needs one (on its stream, synchronously, under the registry's lock: a few ms since they are built by
// additions), freed with the last. A node's ingest queue and its batch contexts hold one 872 MB + 67 MB pair per device
// instead of one each. The ladder's 24-bit tables (key kLadderKey, every GPU context) are shared the same way.
struct SharedBComb {
  int device, bits;
  int4* p;
  int refs;
};
std::mutex g_bcomb_mu;
std::vector<SharedBComb>& bcomb_registry() {
  static std::vector<SharedBComb> r;
  return r;
}

hipError_t bcomb_acquire(int device, int bits, hipStream_t st, const int4** out) {
  std::lock_guard<std::mutex> lk(g_bcomb_mu);
  for (SharedBComb& b : bcomb_registry())
    if (b.device == device && b.bits == bits) {
      ++b.refs;
      *out = b.p;
      return hipSuccess;
    }
  int4* p = nullptr;
  void* scratch = nullptr;
  const bool ladder = bits == kLadderKey;
  hipError_t e = hipMalloc((void**)&p, ladder ? at2v::ladder_btab_bytes() : at2v::bcomb_bytes(bits));
  if (e == hipSuccess) e = hipMalloc(&scratch, at2v::bcomb_scratch_bytes());
#if AT2V_EXP_BCOMB_NOBUILD  // EXPERIMENT (wrong verdicts on the hit path): the hit-list table allocated but never written
  const bool build = ladder || bits == at2v::bcomb_lat_bits();
#else
  const bool build = true;
#endif
  if (e == hipSuccess && build)
    e = ladder ? at2v::launch_build_ladder_btab(p, scratch, st) : at2v::launch_build_bcomb(p, bits, scratch, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (scratch) (void)hipFree(scratch);
  if (e != hipSuccess) {
    if (p) (void)hipFree(p);
    return e;
  }
  bcomb_registry().push_back({device, bits, p, 1});
  *out = p;
  return hipSuccess;
}

void bcomb_release(const int4* p) {
  if (!p) return;
  std::lock_guard<std::mutex> lk(g_bcomb_mu);
  std::vector<SharedBComb>& r = bcomb_registry();
  for (size_t i = 0; i < r.size(); ++i)
    if (r[i].p == p) {
      if (--r[i].refs == 0) {
        (void)hipFree(r[i].p);
        r.erase(r.begin() + (long)i);
      }
      return;
    }
}

void free_cache(SenderCache*& c) {
  if (!c) return;
  if (c->build) (void)hipStreamSynchronize(c->build);  // (the shard's stream: destroyed with the shard)
  for (DevBuf* b : {&c->tags[0], &c->tags[1], &c->entries[0], &c->entries[1], &c->payload, &c->free_slots, &c->used,
                    &c->ctl, &c->seen})
    b->release();
  bcomb_release(c->bcomb);
  bcomb_release(c->bcomb_lat);
  for (DevBuf& b : c->claim_list) b.release();
  if (c->built) (void)hipEventDestroy(c->built);
  if (c->compacted) (void)hipEventDestroy(c->compacted);
  if (c->host_ctl) (void)hipHostFree(c->host_ctl);
  if (c->ctl_copied) (void)hipEventDestroy(c->ctl_copied);
  for (int j = 0; j < kClaimSlots; ++j) {
    if (c->claims_ready[j]) (void)hipEventDestroy(c->claims_ready[j]);
    if (c->slot_free[j]) (void)hipEventDestroy(c->slot_free[j]);
  }
  delete c;
  c = nullptr;
}

// Per-sender cache for `capacity` distinct keys on the current device: 2x as many tag slots (open addressing at
// load <= 1/2), one payload per key. AT2V_TEST_CACHE_FP_BITS (tests only) keeps that many fingerprint bits, so distinct
// keys collide and the byte comparison in the verify kernels is exercised.
int init_cache(Shard& s, uint32_t capacity, uint64_t seed, bool comb, bool admit_first, bool bcomb_wide) {
  SenderCache* c = new (std::nothrow) SenderCache;
  if (!c) return AT2V_E_OOM;
  s.cache = c;
  if (capacity > (1u << 24)) capacity = 1u << 24;
  uint32_t cap = 1024;
  while (cap < 2ull * capacity) cap <<= 1;
  at2v::CacheArgs& a = c->args;
  a.cap = cap;
  a.capacity = capacity;
  a.seed = seed;
  a.fp_mask = ~0ull;
  a.comb = comb ? 1 : 0;
  a.admit_first = admit_first ? 1 : 0;
  // the sighting filter: 2^21 fingerprints (16 MB), so a key seen twice within ~a million records is still found
  a.seen_mask = (1u << 21) - 1;
  if (const char* b = at2v::test_env("AT2V_TEST_CACHE_FP_BITS")) {
    const int bits = std::atoi(b);
    if (bits > 0 && bits < 64) a.fp_mask = (1ull << bits) - 1ull;
  }
  const size_t ctl_bytes = (size_t)at2v::cache_ctl_words() * 8;
  for (int t = 0; t < 2; ++t) {
    AT2V_TRY(c->tags[t].ensure((size_t)cap * 8));
    AT2V_TRY(c->entries[t].ensure((size_t)cap * at2v::cache_entry_bytes()));
    // (on the shard's stream, as every other operation of a context: a process that never touches the null stream maps
    // one hardware queue less)
    AT2V_TRY(hipMemsetAsync(c->tags[t].p, 0, c->tags[t].cap, s.stream));
    AT2V_TRY(hipMemsetAsync(c->entries[t].p, 0, c->entries[t].cap, s.stream));  // every entry invalid
  }
  AT2V_TRY(c->payload.ensure((size_t)capacity * at2v::cache_payload_bytes(a.comb)));
  AT2V_TRY(c->free_slots.ensure((size_t)capacity * 4));
  AT2V_TRY(c->used.ensure((size_t)capacity * 4));
  AT2V_TRY(c->ctl.ensure(ctl_bytes));
  AT2V_TRY(hipMemsetAsync(c->ctl.p, 0, c->ctl.cap, s.stream));
  AT2V_TRY(c->seen.ensure(((size_t)a.seen_mask + 1) * 8));
  AT2V_TRY(hipMemsetAsync(c->seen.p, 0, c->seen.cap, s.stream));
  for (int j = 0; j < kClaimSlots; ++j) AT2V_TRY(c->claim_list[j].ensure((size_t)capacity * 16));
  a.tags = (unsigned long long*)c->tags[0].p;
  a.entries = (int4*)c->entries[0].p;
  a.payload = (int4*)c->payload.p;
  a.free_slots = (uint32_t*)c->free_slots.p;
  a.ctl = (unsigned long long*)c->ctl.p;
  a.seen = (unsigned long long*)c->seen.p;
  a.new_list = (uint4*)c->claim_list[0].p;
  if (comb) {  // the combs of B, built once: 16-bit windows (low-latency kernel and every other comb path) and 20-bit
               // ones for the hit-list kernel, 24-bit with AT2V_CTX_BCOMB_WIDE
    const int lat_bits = at2v::bcomb_lat_bits();
    const int bits = bcomb_wide ? at2v::bcomb_wide_bits() : at2v::bcomb_mid_bits();
    AT2V_TRY(bcomb_acquire(s.device, lat_bits, s.stream, &c->bcomb_lat));
    AT2V_TRY(bcomb_acquire(s.device, bits, s.stream, &c->bcomb));
    a.bcomb_lat = c->bcomb_lat;
    a.bcomb = c->bcomb;
    a.bcomb_bits = bits;
  }
  AT2V_TRY(at2v::launch_cache_init(a, s.stream));
  AT2V_TRY(hipStreamSynchronize(s.stream));
  AT2V_TRY(hipHostMalloc((void**)&c->host_ctl, c->ctl.cap, hipHostMallocDefault));
  std::memset(c->host_ctl, 0, c->ctl.cap);
  c->build = s.stream;
  AT2V_TRY(hipEventCreateWithFlags(&c->ctl_copied, hipEventDisableTiming));
  for (int j = 0; j < kClaimSlots; ++j) {  // recorded once, so the first waits are no-ops
    AT2V_TRY(hipEventCreateWithFlags(&c->claims_ready[j], hipEventDisableTiming));
    AT2V_TRY(hipEventCreateWithFlags(&c->slot_free[j], hipEventDisableTiming));
    AT2V_TRY(hipEventRecord(c->claims_ready[j], s.stream));
    AT2V_TRY(hipEventRecord(c->slot_free[j], c->build));
  }
  AT2V_TRY(hipEventCreateWithFlags(&c->built, hipEventDisableTiming));
  AT2V_TRY(hipEventRecord(c->built, c->build));
  AT2V_TRY(hipEventCreateWithFlags(&c->compacted, hipEventDisableTiming));
  AT2V_TRY(hipEventRecord(c->compacted, c->build));
  return AT2V_OK;
}

// Before a cached launch on `stream`: wait until the launch's claim slot is free; if an earlier launch found the cache
// full (its counters' copy has landed), enqueue a compaction on the build stream, behind every launch and build issued
// so far. Launches issued while it runs look keys up in the old table and claim nothing (CacheArgs::no_claim), so they
// neither wait for it nor touch what it rebuilds (the free list, the spare table). The first launch after it has
// completed swaps the tables in; from then on the build stream also waits for every launch issued before the swap, so a
// payload an evicted entry still held (maybe read by a lookup-only launch) is rebuilt for another key only once those
// launches are done.
hipError_t cache_before_launch(SenderCache& c, Shard& s, hipStream_t stream, int j) {
  hipError_t e = hipStreamWaitEvent(stream, c.slot_free[j], 0);
  if (e == hipSuccess && c.copy_pending && hipEventQuery(c.ctl_copied) == hipSuccess) {
    c.copy_pending = false;
    if (c.host_ctl[at2v::kCtlCompactions] > c.compactions_seen) {  // a compaction has run since the last look
      c.compactions_seen = c.host_ctl[at2v::kCtlCompactions];
      if (c.host_ctl[at2v::kCtlThreshold] == 0) {
        c.freeze_len = c.freeze_len ? std::min<uint32_t>(2 * c.freeze_len, 256) : 8;
        c.freeze_left = c.freeze_len;
      } else {
        c.freeze_len = 0;
      }
    }
    if (c.host_ctl[at2v::kCtlFull] && !c.freeze_left) c.compact_pending = true;
  }
  auto wait_all_launches = [&](hipStream_t st) {  // every launch so far: the last one on each scratch set
    hipError_t r = hipSuccess;
    for (int k = 0; k < s.sets && r == hipSuccess; ++k) r = hipStreamWaitEvent(st, s.scratch_free[k], 0);
    return r;
  };
  if (e == hipSuccess && c.compacting && hipEventQuery(c.compacted) == hipSuccess) {
    e = wait_all_launches(c.build);
    if (e == hipSuccess) {
      const int nx = c.cur ^ 1;
      c.cur = nx;
      c.args.tags = (unsigned long long*)c.tags[nx].p;
      c.args.entries = (int4*)c.entries[nx].p;
      c.compacting = false;
    }
  }
  if (e == hipSuccess && c.compact_pending && !c.compacting) {
    e = wait_all_launches(c.build);  // (the builds before it are on the build stream already)
    const int nx = c.cur ^ 1;
    at2v::CacheCompactArgs x{(unsigned long long*)c.tags[nx].p, (int4*)c.entries[nx].p, (uint32_t*)c.used.p};
    if (e == hipSuccess) e = at2v::launch_cache_compact(c.args, x, c.build);
    if (e == hipSuccess) e = hipEventRecord(c.compacted, c.build);
    if (e == hipSuccess) {
      c.compacting = true;
      c.compact_pending = false;
    }
  }
  c.args.no_claim = c.compacting || c.freeze_left ? 1 : 0;
  if (c.freeze_left) --c.freeze_left;
  return e;
}

// The builds of a cached launch's claim slot (build stream: after the launch, payloads, flip, slot free), then the
// counters' copy for the host (the compaction check of a later launch reads kCtlFull from it): on the context's stream,
// so the caller's stream carries only the verify kernel.
hipError_t enqueue_cache_build(SenderCache& c, const PendingBuild& b) {
  hipError_t e = hipStreamWaitEvent(c.build, c.claims_ready[b.slot], 0);
  if (e == hipSuccess) e = at2v::launch_cache_build(b.args, b.max_claims, c.build);
  if (e == hipSuccess) e = hipEventRecord(c.slot_free[b.slot], c.build);
  if (e == hipSuccess) e = hipEventRecord(c.built, c.build);
  // A new copy only once the host has seen the previous one: re-recording the event behind every launch's builds would
  // keep it "not ready" for as long as launches arrive faster than the build stream drains, and the host would never
  // learn that the cache is full (compaction starved; the counters it reads may be a few launches old instead).
  if (e == hipSuccess && !c.copy_pending) {
    e = hipMemcpyAsync(c.host_ctl, c.ctl.p, c.ctl.cap, hipMemcpyDeviceToHost, c.build);
    if (e == hipSuccess) e = hipEventRecord(c.ctl_copied, c.build);
    c.copy_pending = e == hipSuccess;
  }
  return e;
}

bool scratch_ok(const Shard& s) {
  for (int j = 0; j < s.sets; ++j)
    if (!s.scratch[j].p) return false;
  return s.btab.p != nullptr;
}

// One verify launch on shard s (current device = s.device), on `stream`. The launch takes the shard's next scratch set
// and waits for the launch that last used that set, on whatever stream that ran; launches on different streams may
// therefore run concurrently (on one stream they are ordered anyway). Cached launches may overlap too: they share the tag
// table through atomics, each has its own claim slot (and waits for that slot's previous builds), and every cached launch
// after a compaction waits for it (cache_before_launch). The verdict words are zeroed first (fail closed).
hipError_t launch_shard(at2v_ctx* ctx, Shard& s, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg,
                        uint32_t msg_bytes, const uint32_t* off, uint32_t n, uint32_t* verdicts, hipStream_t stream,
                        bool zero_verdicts = true, bool pipeline = false, const at2v::StagedArgs* staged = nullptr) {
  // a chunk of the host-buffer pipeline whose batch is above small_batch_max: the throughput kernels at every chunk
  // size, with dense grids (launch_verify)
  const uint32_t pair_max = pipeline ? 0u : ctx->pair_max;
  if (!verdicts || (!pk && !staged) || !scratch_ok(s)) return hipErrorInvalidValue;  // (never launch on a null buffer)
  if (ctx->test_fail_launches) {  // test hook: a launch failure, as a faulting device would report it
    --ctx->test_fail_launches;
    return hipErrorLaunchFailure;
  }
  const int j = (int)(s.next_set++ % (unsigned)s.sets);
  hipError_t e = hipStreamWaitEvent(stream, s.scratch_free[j], 0);
  // the cache serves the throughput kernel (launches above small_batch_max records; with combs, every launch)
  SenderCache* c = (s.cache && (n > pair_max || s.cache->args.comb)) ? s.cache : nullptr;
  // the four-wave comb kernel of small batches writes every verdict word of the launch whatever the verdicts (its
  // blocks stride over all chunks), so the zeroing is left out there: one dependent memset less on the latency path
  if (c && c->args.comb && n <= pair_max) zero_verdicts = false;
  if (e == hipSuccess && zero_verdicts) e = hipMemsetAsync(verdicts, 0, ((size_t)n + 31) / 32 * 4, stream);
  const int cs = c ? (int)(c->launches % kClaimSlots) : 0;
  if (e == hipSuccess && c) e = cache_before_launch(*c, s, stream, cs);
  at2v::CacheArgs ca{};
  if (c) {
    c->args.count_word = at2v::kCtlClaims0 + cs;
    c->args.new_list = (uint4*)c->claim_list[cs].p;
    c->args.epoch = (uint32_t)++c->launches;
    ca = c->args;
  }
  at2v::PartArgs pa{};
  const bool part = c && ctx->partition && n > pair_max;
  if (e == hipSuccess && part) {
    const size_t need = (size_t)n * at2v::part_bytes_per_record();
    if (s.part[j].cap < need) {  // grows: the set's previous launch (it reads the old lists) must be done first
      e = hipEventSynchronize(s.scratch_free[j]);
      if (e == hipSuccess) e = s.part[j].ensure(need);
    }
    uint32_t* base = (uint32_t*)s.part[j].p;
    pa = at2v::PartArgs{base, base + n, base + 2 * (size_t)n, nullptr};
  }
  if (e == hipSuccess)
    e = at2v::launch_verify(pk, sig, msg, msg_bytes, off, n, (int)ctx->policy, verdicts, (int4*)s.scratch[j].p,
                            (const int4*)s.btab.p, s.btab24, s.grid, pair_max, stream, c ? &ca : nullptr,
                            part ? &pa : nullptr, pipeline ? 1 : 0, staged);
  if (e == hipSuccess && c) {
    // claims of this launch -> payloads on the build stream (later launches use them; this one did not wait)
    e = hipEventRecord(c->claims_ready[cs], stream);
    if (e == hipSuccess) e = enqueue_cache_build(*c, PendingBuild{ca, std::min(n, ca.capacity), cs});
  }
  if (e == hipSuccess) e = hipEventRecord(s.scratch_free[j], stream);
  return e;
}

// ---- the host-buffer path: chunked, pipelined staging (HostPipe above) ----

hipError_t wait_uploads(StageSlot& sl);

void free_pipe(Shard& s) {
  HostPipe* p = s.pipe;
  if (!p) return;
  for (StageSlot& sl : p->slot)  // (uploads still in flight: a call that failed between submit and launch)
    if (sl.uploaded.handle) (void)wait_uploads(sl);
  for (hipStream_t st : {p->copy, p->comp[0], p->comp[1]})
    if (st) (void)hipStreamSynchronize(st);
  for (StageSlot& sl : p->slot) {
    if (sl.host) (void)hipHostFree(sl.host);
    if (sl.uploaded.handle) (void)hsa_signal_destroy(sl.uploaded);
  }
  if (p->ctl) (void)hipHostFree(p->ctl);
  for (DevBuf& b : p->arenas) b.release();
  for (hipEvent_t ev : p->comp_done)
    if (ev) (void)hipEventDestroy(ev);
  for (hipStream_t st : {p->copy, p->comp[0], p->comp[1]})
    if (st) (void)hipStreamDestroy(st);
  delete p;
  s.pipe = nullptr;
}

hipError_t hsa_err(hsa_status_t st) { return st == HSA_STATUS_SUCCESS ? hipSuccess : hipErrorUnknown; }

hsa_status_t find_cpu_agent(hsa_agent_t a, void* data) {
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_CPU) {
    *static_cast<hsa_agent_t*>(data) = a;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

// A compute stream of the pipe. The two should sit on different hardware queues, or their launches run one after the
// other and every chunk pays its own end-of-launch drain: HIP maps streams onto GPU_MAX_HW_QUEUES (4) shared queues, and
// in a process with a few streams already the two new ones can land on the same queue (profiles/r06/r06d: queue 4 for
// both). mode 0 (default): plain streams; 1: the second one at the highest priority (a queue of its own priority level);
// 2: streams with a full CU mask (HIP gives a CU-masked stream a queue of its own). Test hook AT2V_TEST_PIPE_STREAMS.
// Mode 1 was the default until the end of round 6: the high-priority queues stay with the process after their streams
// are gone, and other processes on the GPU paid for them. Config 5 with a polluter process, run by a pytest process whose
// earlier tests had used 8-shard host-buffer contexts: node queue p99 0.72-1.04 ms with mode 1, 0.48-0.60 ms with mode 0
// (profiles/r06/r06ab, r06ad, r06ae). In a process with few streams the two modes run a 1M-record call alike (r06aa).
hipError_t create_comp_stream(hipStream_t* st, int j, int mode, int device) {
  if (mode == 1 && j == 1) {
    int least = 0, greatest = 0;
    hipError_t e = hipDeviceGetStreamPriorityRange(&least, &greatest);
    return e == hipSuccess ? hipStreamCreateWithPriority(st, hipStreamNonBlocking, greatest) : e;
  }
  if (mode == 2) {
    hipDeviceProp_t prop;
    hipError_t e = hipGetDeviceProperties(&prop, device);
    if (e != hipSuccess) return e;
    std::vector<uint32_t> mask((size_t)(prop.multiProcessorCount + 31) / 32, 0xffffffffu);
    return hipExtStreamCreateWithCUMask(st, (uint32_t)mask.size(), mask.data());
  }
  return hipStreamCreateWithFlags(st, hipStreamNonBlocking);
}

// the shard's pipe (current device = s.device); its events are recorded once, so the first waits are no-ops
hipError_t ensure_pipe(Shard& s, int mode) {
  if (s.pipe) return hipSuccess;
  HostPipe* p = new (std::nothrow) HostPipe;
  if (!p) return hipErrorOutOfMemory;
  s.pipe = p;
  hipError_t e = hipStreamCreateWithFlags(&p->copy, hipStreamNonBlocking);
  for (int j = 0; j < 2 && e == hipSuccess; ++j) {
    e = create_comp_stream(&p->comp[j], j, mode, s.device);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&p->comp_done[j], hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventRecord(p->comp_done[j], p->copy);
  }
  // The uploads go to the DMA engines through HSA directly (a host-to-device hsa_amd_memory_async_copy runs on an SDMA
  // engine): HIP's hipMemcpyAsync handed some of them to blit kernels, which take CUs from the running verify launches
  // and delay the next one (profiles/r06/r06k, r06m: 1.25 ms for a 13 MB upload beside a launch, against 0.23 ms on SDMA).
  // HIP already initialised the runtime; hsa_init only takes a reference.
  if (e == hipSuccess) e = hsa_err(hsa_init());
  if (e == hipSuccess) {
    hsa_amd_pointer_info_t info;
    std::memset(&info, 0, sizeof info);
    info.size = sizeof info;
    e = hsa_err(hsa_amd_pointer_info(s.btab.p, &info, nullptr, nullptr, nullptr));
    if (e == hipSuccess) p->gpu = info.agentOwner;
    if (e == hipSuccess && (hsa_iterate_agents(find_cpu_agent, &p->cpu) != HSA_STATUS_INFO_BREAK || !p->cpu.handle))
      e = hipErrorUnknown;
  }
  for (StageSlot& sl : p->slot)
    if (e == hipSuccess) e = hsa_err(hsa_signal_create(0, 0, nullptr, &sl.uploaded));
  if (e == hipSuccess)
    e = hipHostMalloc((void**)&p->ctl, sizeof(StagedCtl), hipHostMallocCoherent | hipHostMallocMapped);
  if (e == hipSuccess) {
    p->ctl->ready = 0;
    p->ctl->timeout = 0;
  }
  if (e != hipSuccess) free_pipe(s);
  return e;
}

// A staged chunk of c records with mb message bytes: pk | sig | offsets (c + 1, rebased) | messages (+16 bytes of slack
// for the kernels' last-word reads), every part 16-byte aligned.
struct ChunkLayout {
  size_t sig, off, msg, upload, total;
};
ChunkLayout chunk_layout(size_t c, size_t mb) {
  ChunkLayout l;
  l.sig = c * 32;
  l.off = c * 96;
  l.msg = (l.off + (c + 1) * 4 + 15) & ~(size_t)15;
  l.upload = l.msg + mb;
  l.total = l.upload + 16;
  return l;
}

// The host copy of one chunk, split into pieces of about kCopyPiece bytes for the copy pool.
struct CopyPiece {
  uint8_t* dst;
  const uint8_t* src;  // bytes, or (offsets piece) the caller's msg_off + first record
  size_t len;          // bytes, or offsets
  uint32_t base;       // offsets piece: subtracted from every offset
  bool offsets;
};
struct CopyJob {
  std::vector<CopyPiece> pieces;
  void add(uint8_t* dst, const uint8_t* src, size_t len) {
    for (size_t o = 0; o < len; o += kCopyPiece)
      pieces.push_back({dst + o, src + o, std::min(kCopyPiece, len - o), 0, false});
  }
  void add_offsets(uint32_t* dst, const uint32_t* src, size_t count, uint32_t base) {
    const size_t step = kCopyPiece / 4;
    for (size_t o = 0; o < count; o += step)
      pieces.push_back({(uint8_t*)(dst + o), (const uint8_t*)(src + o), std::min(step, count - o), base, true});
  }
  size_t base = 0;  // run_copy: the first piece of the batch the pool is running
  static void run_piece(void* a, size_t i) {
    CopyJob* j = static_cast<CopyJob*>(a);
    const CopyPiece& p = j->pieces[j->base + i];
    if (!p.offsets) {
      std::memcpy(p.dst, p.src, p.len);
      return;
    }
    const uint32_t* s = (const uint32_t*)p.src;
    uint32_t* d = (uint32_t*)p.dst;
    for (size_t k = 0; k < p.len; ++k) d[k] = s[k] - p.base;
  }
};

// Records [a, a + c) of the caller's batch (absolute indices; a multiple of 64 relative to the shard's first record, so
// the chunk owns whole verdict words) -> staging slot -> device -> verify launch writing d_words (the chunk's words of
// the shard's device bitmap, zeroed by the launch first). Current device = s.device. Returns after the launch is
// enqueued; the host waits only for the slot's previous upload (and, when the slot must grow, for its previous launch).
// Host copy of one job (the copy pool's threads for large ones, the calling thread for small ones).
// The pieces go in batches of kCopyBatch; `between` runs after each batch (issue_chunk: launch the previous chunk as soon
// as its uploads are done, not only after this whole copy).
template <class Between>
void run_copy(at2v::CpuPool* copier, CopyJob& job, size_t bytes, Between&& between) {
  const size_t np = job.pieces.size();
  for (job.base = 0; job.base < np; job.base += kCopyBatch) {
    const size_t cnt = std::min(kCopyBatch, np - job.base);
    if (copier && bytes >= kCopyPoolMin) {
      at2v::pool_run(copier, cnt, CopyJob::run_piece, &job);
    } else {
      for (size_t i = 0; i < cnt; ++i) CopyJob::run_piece(&job, i);
    }
    between();
  }
  job.pieces.clear();
  job.base = 0;
}

// device bytes a shard's part of a host batch takes in the pipe's arena: every chunk's layout, 256-aligned
size_t arena_bytes(size_t m, size_t mb, size_t first) {
  const size_t chunks = m / (first ? first : 1) + 2;
  return m * 100 + mb + chunks * (16 + 4 + 16 + 256) + 256;
}

// wait for a slot's uploads (an SDMA error leaves the signal negative). Bounded: uploads that have not landed after
// kUploadWaitS fail the call instead of hanging it.
constexpr double kUploadWaitS = 10.0;
hipError_t wait_uploads(StageSlot& sl) {
  static const uint64_t hint = [] {  // ~1 ms in HSA timestamp ticks (the wait below re-checks the deadline)
    uint64_t f = 0;
    return hsa_system_get_info(HSA_SYSTEM_INFO_TIMESTAMP_FREQUENCY, &f) == HSA_STATUS_SUCCESS && f ? f / 1000 : 100000;
  }();
  const auto t0 = std::chrono::steady_clock::now();
  hsa_signal_value_t v;
  while ((v = hsa_signal_wait_scacquire(sl.uploaded, HSA_SIGNAL_CONDITION_LT, 1, hint, HSA_WAIT_STATE_ACTIVE)) > 0)
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > kUploadWaitS)
      return hipErrorLaunchTimeOut;
  if (v == 0) return hipSuccess;
  hsa_signal_store_screlease(sl.uploaded, 0);  // (reported once; the slot starts clean for the next call)
  return hipErrorUnknown;
}

// The launch of the shard's pending chunk (current device = s.device), once its uploads are done: the launch needs no
// device-side dependency on the copies, so the verify kernels run back to back on the compute streams while the host
// stages the next chunks.
hipError_t flush_chunk(at2v_ctx* ctx, Shard& s) {
  HostPipe& p = *s.pipe;
  if (!p.pending) return hipSuccess;
  p.pending = false;
  const ChunkLaunch& k = p.pend;
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  hipError_t e = wait_uploads(p.slot[k.slot]);
  if (ctx->pipe_trace) ctx->tr_wait += std::chrono::duration<double>(clk::now() - t0).count();
  if (e == hipSuccess)
    e = launch_shard(ctx, s, k.d, k.d + k.sig, k.d + k.msg, (uint32_t)k.mb, (const uint32_t*)(k.d + k.off),
                     (uint32_t)k.c, k.d_words, p.comp[k.stream], true, k.throughput);
  if (e == hipSuccess) e = hipEventRecord(p.comp_done[k.stream], p.comp[k.stream]);
  return e;
}

// Records [a, a + c) of the caller's batch (absolute indices; a multiple of 64 relative to the shard's first record, so
// the chunk owns whole verdict words): staging slot -> DMA uploads into the chunk's own region of the pipe's device
// arena -> (the next call of this function, or flush_chunk) verify launch writing d_words (the chunk's words of the
// shard's device bitmap, zeroed by the launch first). Current device = s.device. The four parts (pk, sig + offsets,
// messages) are copied and submitted one after the other, so the DMA of one overlaps the host copy of the next; then the
// previous chunk is launched (its uploads had this chunk's host copy to finish). The first chunk of a call (`first`)
// is launched at once: it is the pipeline's fill.
hipError_t issue_chunk(at2v_ctx* ctx, Shard& s, at2v::CpuPool* copier, const uint8_t* pk, const uint8_t* sig,
                       const uint8_t* msg, const uint32_t* msg_off, size_t a, size_t c, uint32_t* d_words,
                       bool throughput, bool first) {
  HostPipe& p = *s.pipe;
  const int k = (int)(p.chunks % kStageSlots);
  StageSlot& sl = p.slot[k];
  const uint32_t mb0 = msg_off[a];
  const size_t mb = (size_t)(msg_off[a + c] - mb0);
  const ChunkLayout L = chunk_layout(c, mb);
  if (p.arena_at + L.total > p.arena().cap) return hipErrorInvalidValue;  // (sized by the caller: cannot happen)
  uint8_t* d = (uint8_t*)p.arena().p + p.arena_at;
  p.arena_at += (L.total + 255) & ~(size_t)255;
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  hipError_t e = wait_uploads(sl);  // (done already: the slot's chunk was launched, which waited for them)
  if (e == hipSuccess && sl.host_cap < L.total) {
    if (sl.host) (void)hipHostFree(sl.host);
    sl.host = nullptr;
    sl.host_cap = 0;
    const size_t want = std::max(L.total + L.total / 4, chunk_layout(ctx->stage_max, 0).total);
    e = hipHostMalloc((void**)&sl.host, want, hipHostMallocDefault);
    if (e == hipSuccess) sl.host_cap = want;
  }
  if (e != hipSuccess) return e;
  const auto t1 = clk::now();
  hsa_signal_store_screlease(sl.uploaded, mb ? 3 : 2);  // the parts below, each decrements it when done
  auto upload = [&](size_t at, size_t len) {
    return hsa_err(hsa_amd_memory_async_copy(d + at, p.gpu, sl.host + at, p.cpu, len, 0, nullptr, sl.uploaded));
  };
  // between copy batches: the pending (previous) chunk is launched as soon as its uploads have landed, so the device
  // does not wait for this chunk's whole host copy (the pipeline's fill: the second chunk's launch)
  hipError_t ef = hipSuccess;
  auto poll = [&]() {
    if (ef == hipSuccess && p.pending && hsa_signal_load_scacquire(p.slot[p.pend.slot].uploaded) == 0)
      ef = flush_chunk(ctx, s);
  };
  CopyJob job;
  job.add(sl.host, pk + a * 32, c * 32);
  run_copy(copier, job, c * 32, poll);
  e = upload(0, c * 32);
  job.add(sl.host + L.sig, sig + a * 64, c * 64);
  job.add_offsets((uint32_t*)(sl.host + L.off), msg_off + a, c + 1, mb0);
  run_copy(copier, job, c * 68, poll);
  if (e == hipSuccess) e = upload(L.sig, L.msg - L.sig);
  if (mb) {
    job.add(sl.host + L.msg, msg + mb0, mb);
    run_copy(copier, job, mb, poll);
    if (e == hipSuccess) e = upload(L.msg, mb);
  }
  if (e == hipSuccess) e = ef;
  if (e != hipSuccess) {  // (a submit failed: nothing waits for this slot's parts any more; the call fails)
    hsa_signal_store_screlease(sl.uploaded, 0);
    return e;
  }
  const auto t2 = clk::now();
  e = flush_chunk(ctx, s);
  p.pend = ChunkLaunch{d, L.sig, L.off, L.msg, mb, c, d_words, throughput, k, (int)(p.chunks % 2)};
  p.pending = true;
  if (e == hipSuccess && first) e = flush_chunk(ctx, s);
  ++p.chunks;
  ++ctx->host_chunks;
  if (ctx->pipe_trace) {
    const auto t3 = clk::now();
    ctx->tr_wait += std::chrono::duration<double>(t1 - t0).count();
    ctx->tr_copy += std::chrono::duration<double>(t2 - t1).count();
    ctx->tr_enq += std::chrono::duration<double>(t3 - t2).count();
  }
  return e;
}

// ---- the staged form (StagedPlan above) ----

void stage_store(HostPipe& p, uint32_t count) {
  __atomic_store_n(&p.ctl->ready, ((unsigned long long)p.epoch << 32) | count, __ATOMIC_RELEASE);
}

// Publish the regions whose uploads have landed, in order: those below `block_below` are waited for, later ones only if
// already done. An upload error (negative signal) is returned; the caller aborts.
hipError_t stage_publish(HostPipe& p, StagedPlan& sp, uint32_t block_below) {
  const uint32_t before = sp.published;
  hipError_t e = hipSuccess;
  while (sp.published < sp.submitted) {
    StageSlot& sl = p.slot[sp.published % kStageSlots];
    if (sp.published >= block_below && hsa_signal_load_scacquire(sl.uploaded) > 0) break;
    e = wait_uploads(sl);
    if (e != hipSuccess) break;
    ++sp.published;
  }
  if (sp.published != before) stage_store(p, sp.published);
  return e;
}

// the single launch of a staged call, on comp[0]
hipError_t stage_launch(at2v_ctx* ctx, Shard& s, StagedPlan& sp) {
  HostPipe& p = *s.pipe;
  const at2v::StagedArgs& sa = sp.args;
  const size_t m = sp.m;
  hipError_t e = launch_shard(ctx, s, (const uint8_t*)p.arena().p, nullptr, nullptr, 0, nullptr, (uint32_t)m,
                              sp.verdicts, p.comp[0], /*zero_verdicts=*/false, /*pipeline=*/true, &sa);
  if (e == hipSuccess) e = hipEventRecord(p.comp_done[0], p.comp[0]);
  if (e != hipSuccess) sp.active = false;  // (nothing launched: nobody waits for the word)
  sp.launched = e == hipSuccess;
  return e;
}

// The call's launch for shard s (current device = s.device): layout of the regions in the arena, then the single launch
// on comp[0]; its waves wait for the regions the host publishes.
hipError_t stage_begin(at2v_ctx* ctx, Shard& s, StagedPlan& sp, size_t lo, size_t m, const uint32_t* msg_off,
                       uint32_t* d_verdicts) {
  HostPipe& p = *s.pipe;
  for (StageSlot& sl : p.slot) (void)wait_uploads(sl);  // (after a failed call, uploads may still write the arena)
  p.pending = false;
  sp = StagedPlan{};
  sp.active = true;
  sp.verdicts = d_verdicts;
  sp.lo = lo;
  sp.m = m;
  sp.ushift = kStageRegionMinLog2;
  while (((m + ((size_t)1 << sp.ushift) - 1) >> sp.ushift) > (size_t)at2v::kMaxStageRegions) ++sp.ushift;
  const size_t U = (size_t)1 << sp.ushift;
  sp.nreg = (uint32_t)((m + U - 1) / U);
  at2v::StagedArgs sa{};
  size_t total = 0;
  sp.at.resize(sp.nreg);
  for (uint32_t u = 0; u < sp.nreg; ++u) {
    const size_t a = lo + u * U, c = std::min(U, m - u * U);
    const size_t mb = (size_t)(msg_off[a + c] - msg_off[a]);
    sp.at[u] = total;
    sa.mb[u] = (uint32_t)mb;
    total += (chunk_layout(c, mb).total + 255) & ~(size_t)255;
  }
  hipError_t e = p.arena().ensure(total);
  if (e != hipSuccess) return e;
  for (uint32_t u = 0; u < sp.nreg; ++u) sa.at[u] = sp.at[u];
  ++p.epoch;
  p.ctl->timeout = 0;
  stage_store(p, 0);
  sa.ready = &p.ctl->ready;
  sa.timeout = &p.ctl->timeout;
  sa.epoch = p.epoch;
  sa.ushift = sp.ushift;
  sa.nreg = sp.nreg;
  sa.last_c = (uint32_t)(m - (size_t)(sp.nreg - 1) * U);
  sa.nap = ctx->stage_nap;
  sp.args = sa;
  if (ctx->stage_pre || ctx->stage_launch_at) return hipSuccess;  // (stage_launch later)
  return stage_launch(ctx, s, sp);
}

// Region u of the plan: host copy into its slot (after the slot's previous region has landed and been published), DMA
// uploads into the arena; between copy batches, the regions that have landed are published. Region 0 is published as
// soon as it lands (the launch's waves are waiting for it).
hipError_t stage_region(at2v_ctx* ctx, Shard& s, at2v::CpuPool* copier, StagedPlan& sp, const uint8_t* pk,
                        const uint8_t* sig, const uint8_t* msg, const uint32_t* msg_off) {
  HostPipe& p = *s.pipe;
  const uint32_t u = sp.submitted;
  const size_t U = (size_t)1 << sp.ushift;
  const size_t a = sp.lo + u * U, c = std::min(U, sp.m - u * U);
  const uint32_t mb0 = msg_off[a];
  const size_t mb = (size_t)(msg_off[a + c] - mb0);
  const ChunkLayout L = chunk_layout(c, mb);
  const int k = (int)(u % kStageSlots);
  StageSlot& sl = p.slot[k];
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  hipError_t e = stage_publish(p, sp, u >= kStageSlots ? u - kStageSlots + 1 : 0);  // the slot's previous region
  if (e == hipSuccess && sl.host_cap < L.total) {
    if (sl.host) (void)hipHostFree(sl.host);
    sl.host = nullptr;
    sl.host_cap = 0;
    const size_t want = std::max(L.total + L.total / 4, chunk_layout(U, 0).total + U * 128);
    e = hipHostMalloc((void**)&sl.host, want, hipHostMallocDefault);
    if (e == hipSuccess) sl.host_cap = want;
  }
  if (e != hipSuccess) return e;
  const auto t1 = clk::now();
  uint8_t* d = (uint8_t*)p.arena().p + sp.at[u];
  hsa_signal_store_screlease(sl.uploaded, mb ? 3 : 2);
  auto upload = [&](size_t at, size_t len) {
    return hsa_err(hsa_amd_memory_async_copy(d + at, p.gpu, sl.host + at, p.cpu, len, 0, nullptr, sl.uploaded));
  };
  hipError_t ep = hipSuccess;
  auto poll = [&]() {
    if (ep == hipSuccess) ep = stage_publish(p, sp, 0);
  };
  CopyJob job;
  job.add(sl.host, pk + a * 32, c * 32);
  run_copy(copier, job, c * 32, poll);
  e = upload(0, c * 32);
  job.add(sl.host + L.sig, sig + a * 64, c * 64);
  job.add_offsets((uint32_t*)(sl.host + L.off), msg_off + a, c + 1, mb0);
  run_copy(copier, job, c * 68, poll);
  if (e == hipSuccess) e = upload(L.sig, L.msg - L.sig);
  if (mb) {
    job.add(sl.host + L.msg, msg + mb0, mb);
    run_copy(copier, job, mb, poll);
    if (e == hipSuccess) e = upload(L.msg, mb);
  }
  if (e != hipSuccess) {
    hsa_signal_store_screlease(sl.uploaded, 0);
    return e;
  }
  sp.submitted = u + 1;
  sp.slot_region[k] = (int)u;
  const auto t2 = clk::now();
  e = ep;
  const uint32_t la = std::min(ctx->stage_launch_at, sp.nreg);
  if (e == hipSuccess) e = stage_publish(p, sp, u == 0 ? 1 : (!ctx->stage_pre && u + 1 == la ? la : 0));
  if (e == hipSuccess && !ctx->stage_pre && !sp.launched && la && sp.published >= la) e = stage_launch(ctx, s, sp);
  ++p.chunks;
  ++ctx->host_chunks;
  if (ctx->pipe_trace) {
    const auto t3 = clk::now();
    ctx->tr_wait += std::chrono::duration<double>(t1 - t0).count() + std::chrono::duration<double>(t3 - t2).count();
    ctx->tr_copy += std::chrono::duration<double>(t2 - t1).count();
  }
  return e;
}

// a failed staged call: the launch's waves stop waiting (their chunks' verdicts are 0; the call reports the error)
void stage_abort(HostPipe& p, StagedPlan& sp) {
  if (sp.active) stage_store(p, 0x80000000u);
}

// The pipe's arena for a shard's part of a call (m records, mb message bytes), before its first chunk: every launch of
// the previous host-buffer call has completed (the call waited for its verdict copy, which followed them).
hipError_t begin_arena(at2v_ctx* ctx, Shard& s, size_t m, size_t mb) {
  HostPipe& p = *s.pipe;
  for (StageSlot& sl : p.slot) (void)wait_uploads(sl);  // (after a failed call, uploads may still write the arena)
  p.pending = false;
  p.arena_at = 0;
  return p.arena().ensure(arena_bytes(m, mb, std::min(ctx->stage_first, std::max<size_t>(m, 1))));
}

// The chunk schedule of one shard's part of a host batch: a part the low-latency kernel takes whole (<= small_batch_max
// records) is one chunk; a larger one starts with kStageFirstRecords (the pipeline's fill: nothing runs on the device until
// it is up), then doubles up to kStageMaxRecords, and a remainder smaller than the first chunk joins the chunk before
// it. Those chunks run the throughput kernels with dense grids whatever their size (launch_shard `pipeline`). Every
// chunk but the last is a multiple of 64 records.
struct ChunkPlan {
  size_t first = 0, next = 0, pos = 0, m = 0, cap = 0;
  void init(size_t m_, const at2v_ctx* ctx) {
    m = m_;
    pos = 0;
    first = m <= ctx->pair_max ? std::max<size_t>(m, 64) : ctx->stage_first;
    cap = std::max(ctx->stage_max, first);
    next = first;
  }
  bool done() const { return pos >= m; }
  size_t take() {  // the next chunk's record count (its first record is pos before the call)
    size_t c = std::min(next, m - pos);
    if (m - pos - c < first) c = m - pos;
    if (pos > 0 || first >= cap) next = std::min(next * 2, cap);  // (the first size twice: two launches fill the device)
    pos += c;
    return c;
  }
};

at2v::CpuPool* copy_pool(at2v_ctx* ctx) {
  if (!ctx->copier && ctx->copy_threads > 1)
    ctx->copier = at2v::copy_pool_create(std::min(ctx->copy_threads, at2v::usable_cpus()));
  return ctx->copier;  // (nullptr: the calling thread copies alone)
}

int nccl_code(ncclResult_t r) { return r == ncclSuccess ? AT2V_OK : AT2V_E_RCCL; }

// AT2V_EXPERIMENT_* bits of this library: the kernels object's switches and this file's
unsigned library_experiments() {
  unsigned m = at2v::kernel_experiments();
#if AT2V_EXP_BCOMB_NOBUILD
  m |= AT2V_EXPERIMENT_BCOMB_NOBUILD;
#endif
  return m;
}

// The collective step of a rank (current device = its shard's): zero this rank's slice `mine` of the node bitmap,
// verify its records into it unless an earlier local step already failed (`local` != AT2V_OK), then ALWAYS join the
// in-place all-gather, so a failure on one rank never leaves the other ranks blocked inside the collective
// (VERDICT r2 "What's weak" 4). A rank that failed contributes zero words: its records are verdict 0 on every rank
// (fail closed). If even the zeroing of its slice failed, it sends the context's all-zero buffer instead. Returns the
// first local error, else the RCCL result.
int gather_shard(at2v_ctx* ctx, Shard& s, int local, const uint8_t* d_pk, const uint8_t* d_sig, const uint8_t* d_msg,
                 size_t msg_bytes, const uint32_t* d_msg_off, size_t n_local, size_t wpr, uint32_t* d_bitmap,
                 hipStream_t st) {
  uint32_t* mine = d_bitmap + (size_t)ctx->rank * wpr;
  // A zero buffer of this call's size exists before any work (it grows, zeroed, on the first call with a larger
  // words_per_rank): a rank that fails anywhere below sends it, never its slice, whose contents are then unknown.
  DevBuf& zb = wpr * 4 <= ctx->zeros.cap ? ctx->zeros : ctx->zeros_big;  // zeros: kGatherWindow words (comm init)
  bool zeros_ok = zb.cap >= wpr * 4;
  if (!zeros_ok) {
    zeros_ok = zb.ensure(wpr * 4) == hipSuccess && hipMemset(zb.p, 0, zb.cap) == hipSuccess;
    if (!zeros_ok) zb.release();
    if (!zeros_ok && local == AT2V_OK) local = AT2V_E_OOM;
  }
  const hipError_t ez = hipMemsetAsync(mine, 0, wpr * 4, st);  // pad words (and an empty rank's whole slice) are 0
  if (ez != hipSuccess && local == AT2V_OK) local = hip_code(ez);
  if (local == AT2V_OK && n_local) {
    const hipError_t e = launch_shard(ctx, s, d_pk, d_sig, d_msg, (uint32_t)msg_bytes, d_msg_off, (uint32_t)n_local,
                                      mine, st, /*zero_verdicts=*/false);
    if (e != hipSuccess) local = hip_code(e);
  }
  // a failed rank contributes zero words (fail closed). Only if it could neither zero its slice nor hold a zero buffer
  // (a device that fails every allocation and memset) does it send its slice as it is.
  const void* send = mine;
  if (local != AT2V_OK && zeros_ok) send = zb.p;
  // Collectives of one communicator run one at a time in issue order on every rank: a caller that alternates streams
  // (so that consecutive verify launches overlap) must not let two all-gathers run concurrently, or ranks could
  // execute them in different orders. This one waits for the previous one, whatever stream it ran on.
  if (ctx->gather_done) (void)hipStreamWaitEvent(st, ctx->gather_done, 0);
  // in place when send == recvbuff + rank * count
  const ncclResult_t r = ncclAllGather(send, d_bitmap, wpr, ncclUint32, ctx->comm, st);
  ++ctx->gathers;
  if (ctx->gather_done) (void)hipEventRecord(ctx->gather_done, st);
  return local != AT2V_OK ? local : nccl_code(r);
}

}  // namespace

extern "C" {

int at2v_create(const at2v_opts* opts, at2v_ctx** out) {
  if (!out) return AT2V_E_INVALID;
  *out = nullptr;
  // a timing-experiment build (wrong verdicts) serves no context unless the process explicitly allows it
  if (library_experiments()) {
    const char* allow = std::getenv("AT2V_ALLOW_EXPERIMENT");
    if (!allow || std::strcmp(allow, "1") != 0) return AT2V_E_INVALID;
  }
  at2v_opts o{0, 1, AT2V_POLICY_DALEK_V1, 0, 0, 0, 0, 0};
  if (opts) o = *opts;
  if (o.num_gpus < 0 || o.num_gpus > 64) return AT2V_E_INVALID;
  if (o.policy != AT2V_POLICY_DALEK_V1 && o.policy != AT2V_POLICY_LIBSODIUM_1_0_18) return AT2V_E_INVALID;
  if (o.flags & ~(AT2V_CTX_CPU_FALLBACK | AT2V_CTX_ADMIT_FIRST | AT2V_CTX_BCOMB_WIDE)) return AT2V_E_INVALID;
  if (o.num_gpus == 0) {  // the CPU batch backend: no HIP call at all
    at2v_ctx* c = new (std::nothrow) at2v_ctx;
    if (!c) return AT2V_E_OOM;
    c->policy = o.policy;
    c->flags = o.flags;
    c->cpu = at2v::cpu_pool_create(o.cpu_threads);
    if (!c->cpu) {
      delete c;
      return AT2V_E_OOM;
    }
    *out = c;
    return AT2V_OK;
  }
  // AT2V_TEST_DEVICE_ALIAS (tests only): shard g runs on device (device + g) % ndev, so a one-GPU box executes the
  // single-process multi-device path (split, per-shard streams, scratch, B tables and caches) with num_gpus > ndev
  const bool alias = at2v::test_env_long("AT2V_TEST_DEVICE_ALIAS", 0) != 0;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return AT2V_E_NODEVICE;
  if (o.device < 0 || o.device >= ndev || (!alias && o.device + o.num_gpus > ndev)) return AT2V_E_NODEVICE;
  at2v_ctx* c = new (std::nothrow) at2v_ctx;
  if (!c) return AT2V_E_OOM;
  c->policy = o.policy;
  c->flags = o.flags;
  c->test_fail_launches = (uint32_t)at2v::test_env_long("AT2V_TEST_FAIL_LAUNCH", 0);
  c->partition = at2v::test_env_long("AT2V_CACHE_PARTITION", 1) != 0;  // (A/B: 0 = round 4)
  c->stage_first = (size_t)at2v::test_env_long("AT2V_TEST_STAGE_FIRST", (long)kStageFirstRecords) / 64 * 64;
  c->stage_max = (size_t)at2v::test_env_long("AT2V_TEST_STAGE_MAX", (long)kStageMaxRecords) / 64 * 64;
  c->copy_threads = (unsigned)at2v::test_env_long("AT2V_TEST_COPY_THREADS", 8);
  c->pipe_streams = (int)at2v::test_env_long("AT2V_TEST_PIPE_STREAMS", c->pipe_streams);
  c->pipe_trace = at2v::test_env_long("AT2V_TEST_PIPE_TRACE", 0) != 0;
  c->staged = at2v::test_env_long("AT2V_TEST_STAGED", 0) != 0;
  c->stage_nap = (uint32_t)at2v::test_env_long("AT2V_TEST_STAGE_NAP", 2);
  c->stage_pre = at2v::test_env_long("AT2V_TEST_STAGE_PRE", 0) != 0;
  c->stage_launch_at = (uint32_t)at2v::test_env_long("AT2V_TEST_STAGE_LAUNCH_AT", 0);
  if (c->stage_first < 64) c->stage_first = 64;
  if (c->stage_max < c->stage_first) c->stage_max = c->stage_first;
  c->pair_max = o.small_batch_max == 0 ? AT2V_SMALL_BATCH_DEFAULT
                : o.small_batch_max == AT2V_SMALL_BATCH_OFF ? 0u : o.small_batch_max;
  c->shards.resize((size_t)o.num_gpus);
  int prev = 0;
  (void)hipGetDevice(&prev);
  std::random_device rd;
  // test hook (A/B runs of processes the caller does not configure, e.g. the config-5 mini-network's nodes)
  const bool wide_env = at2v::test_env_long("AT2V_BCOMB_WIDE", 0) != 0;
  for (int g = 0; g < o.num_gpus; ++g) {
    int rc = init_shard(c->shards[(size_t)g], alias ? (o.device + g) % ndev : o.device + g);
    if (rc == AT2V_OK && o.sender_cache)
      rc = init_cache(c->shards[(size_t)g], o.sender_cache, ((uint64_t)rd() << 32) ^ rd(), o.sender_comb != 0,
                      (o.flags & AT2V_CTX_ADMIT_FIRST) != 0, (o.flags & AT2V_CTX_BCOMB_WIDE) != 0 || wide_env);
    // the cross-rank failure flag of at2v_comm_init_rank / at2v_verify_batch_sharded (first device): allocated here,
    // so a rank whose communicator set-up fails can still join the outcome all-reduce
    if (rc == AT2V_OK && g == 0) rc = hip_code(c->status.ensure(4));
    if (rc == AT2V_OK && g == 0 && (o.flags & AT2V_CTX_CPU_FALLBACK)) {
      c->cpu = at2v::cpu_pool_create(o.cpu_threads);
      if (!c->cpu) rc = AT2V_E_OOM;
    }
    if (rc != AT2V_OK) {
      (void)hipSetDevice(prev);
      at2v_destroy(c);
      return rc;
    }
  }
  (void)hipSetDevice(prev);
  *out = c;
  return AT2V_OK;
}

void at2v_destroy(at2v_ctx* ctx) {
  if (!ctx) return;
  // drain first: the last all-gather may still run on a caller's stream, and verify launches on the
  // shard streams or on callers' streams are ordered before each shard's scratch_free event
  for (Shard& s : ctx->shards) {
    if (hipSetDevice(s.device) != hipSuccess) continue;
    if (s.stream) (void)hipStreamSynchronize(s.stream);
    if (s.pipe)
      for (hipStream_t st : {s.pipe->copy, s.pipe->comp[0], s.pipe->comp[1]}) (void)hipStreamSynchronize(st);
    for (hipEvent_t ev : s.scratch_free)
      if (ev) (void)hipEventSynchronize(ev);
  }
  if (ctx->comm) {
    (void)hipSetDevice(ctx->shards.empty() ? 0 : ctx->shards[0].device);
    if (ctx->gather_done) (void)hipEventSynchronize(ctx->gather_done);
    (void)ncclCommFinalize(ctx->comm);
    (void)ncclCommDestroy(ctx->comm);
    ctx->comm = nullptr;
  }
  if (ctx->gather_done) (void)hipEventDestroy(ctx->gather_done);
  ctx->window.release();
  ctx->zeros.release();
  ctx->zeros_big.release();
  ctx->status.release();
  for (Shard& s : ctx->shards) {
    if (hipSetDevice(s.device) != hipSuccess) continue;
    for (hipEvent_t ev : s.scratch_free)
      if (ev) (void)hipEventDestroy(ev);
    if (s.copied) (void)hipEventDestroy(s.copied);
    for (hipEvent_t ev : s.hcopied)
      if (ev) (void)hipEventDestroy(ev);
    for (DevBuf& b : s.hverdict) b.release();
    free_pipe(s);
    free_cache(s.cache);
    for (DevBuf& b : s.scratch) b.release();
    for (DevBuf& b : s.part) b.release();
    s.btab.release();
    bcomb_release(s.btab24);
    s.pk.release();
    s.sig.release();
    s.msg.release();
    s.off.release();
    s.verdict.release();
    if (s.stream) (void)hipStreamDestroy(s.stream);
  }
  at2v::cpu_pool_destroy(ctx->cpu);
  at2v::cpu_pool_destroy(ctx->copier);
  delete ctx;
}

namespace {

// Issue a host-buffer call into slot k: per shard (64-aligned index range: its words start at word lo/32 of the caller's
// array) the device bitmap and the pipe, then the chunks of all shards round robin, so every device's pipeline fills
// early and the copy pool serves them in turn; then the verdict copies. Returns once everything is enqueued (the host
// copies are done; the launches and downloads run on).
void host_call_issue(at2v_ctx* ctx, int k) {
  HostCall& hc = ctx->calls[k];
  const uint8_t *pk = hc.pk, *sig = hc.sig, *msg = hc.msg;
  const uint32_t* msg_off = hc.msg_off;
  const size_t n = hc.n, G = ctx->shards.size();
  at2v::CpuPool* copier = copy_pool(ctx);
  std::vector<ChunkPlan> plan(G);
  std::vector<StagedPlan> stp(G);
  std::vector<size_t> lo(G);
  std::vector<hipError_t>& err = hc.err;
  err.assign(G, hipSuccess);
  hc.m.assign(G, 0);
  hc.staged.assign(G, 0);
  hc.t0 = std::chrono::steady_clock::now();
  ctx->tr_wait = ctx->tr_copy = ctx->tr_enq = 0;
  for (size_t g = 0; g < G; ++g) {
    Shard& s = ctx->shards[g];
    const at2v::Range r = at2v::device_range(n, G, g);
    lo[g] = r.lo;
    plan[g].init(r.size(), ctx);
    hc.m[g] = r.size();
    if (r.size() == 0) continue;
    hipError_t e = hipSetDevice(s.device);
    if (e == hipSuccess) e = s.hverdict[k].ensure(((r.size() + 31) / 32) * 4);
    if (e == hipSuccess) e = ensure_pipe(s, ctx->pipe_streams);
    if (e == hipSuccess) s.pipe->cur = k;
    if (e == hipSuccess && ctx->staged && !s.cache && r.size() > ctx->pair_max) {
      e = stage_begin(ctx, s, stp[g], r.lo, r.size(), msg_off, (uint32_t*)s.hverdict[k].p);
      hc.staged[g] = 1;
    } else if (e == hipSuccess) {
      e = begin_arena(ctx, s, r.size(), (size_t)(msg_off[r.hi] - msg_off[r.lo]));
    }
    err[g] = e;
  }
  for (bool more = true; more;) {
    more = false;
    for (size_t g = 0; g < G; ++g) {
      if (err[g] != hipSuccess) continue;
      Shard& s = ctx->shards[g];
      if (stp[g].active) {
        StagedPlan& sp = stp[g];
        if (sp.submitted >= sp.nreg) continue;
        err[g] = hipSetDevice(s.device);
        if (err[g] == hipSuccess) err[g] = stage_region(ctx, s, copier, sp, pk, sig, msg, msg_off);
        more = more || sp.submitted < sp.nreg;
        continue;
      }
      ChunkPlan& cp = plan[g];
      if (cp.done()) continue;
      const size_t at = cp.pos, c = cp.take();
      err[g] = hipSetDevice(s.device);
      if (err[g] == hipSuccess)
        err[g] = issue_chunk(ctx, s, copier, pk, sig, msg, msg_off, lo[g] + at, c, (uint32_t*)s.hverdict[k].p + at / 32,
                             cp.m > ctx->pair_max, at == 0);
      more = more || !cp.done();
    }
  }
  for (size_t g = 0; g < G; ++g) {  // the last chunk of every shard / every staged region published
    Shard& s = ctx->shards[g];
    if (plan[g].m == 0 || !s.pipe) continue;
    hipError_t e = hipSetDevice(s.device);
    if (e == hipSuccess && stp[g].active && err[g] == hipSuccess) {
      e = stage_publish(*s.pipe, stp[g], stp[g].submitted);
      if (e == hipSuccess && !stp[g].launched) e = stage_launch(ctx, s, stp[g]);
    } else if (e == hipSuccess && !stp[g].active) {
      e = flush_chunk(ctx, s);
    }
    if (err[g] == hipSuccess) err[g] = e;
    if (err[g] != hipSuccess) stage_abort(*s.pipe, stp[g]);
  }
  // the verdict words of each shard, once its last two launches are done (copy stream)
  for (size_t g = 0; g < G; ++g) {
    Shard& s = ctx->shards[g];
    const size_t m = plan[g].m;
    if (m == 0) continue;
    hipError_t e = err[g];
    if (e == hipSuccess) e = hipSetDevice(s.device);
    HostPipe* p = s.pipe;
    for (int j = 0; j < 2 && e == hipSuccess; ++j) e = hipStreamWaitEvent(p->copy, p->comp_done[j], 0);
    if (e == hipSuccess)
      e = hipMemcpyAsync(hc.verdicts + lo[g] / 32, s.hverdict[k].p, ((m + 31) / 32) * 4, hipMemcpyDeviceToHost,
                         p->copy);
    if (e == hipSuccess) e = hipEventRecord(s.hcopied[k], p->copy);
    err[g] = e;
  }
}

// Complete slot k's call: wait for its verdict copies (not for the cache builds behind them); on a device error with
// AT2V_CTX_CPU_FALLBACK, drain and verify the batch on the CPU (the caller's buffers are still valid: the call has not
// returned to the caller as complete).
void host_call_finish(at2v_ctx* ctx, int k) {
  HostCall& hc = ctx->calls[k];
  if (!hc.active || hc.done) return;
  int rc = AT2V_OK;
  for (size_t g = 0; g < ctx->shards.size(); ++g)
    if (hc.m[g] && hc.err[g] != hipSuccess && rc == AT2V_OK) rc = hip_code(hc.err[g]);
  for (size_t g = 0; g < ctx->shards.size(); ++g) {
    Shard& s = ctx->shards[g];
    if (hc.m[g] == 0 || hc.err[g] != hipSuccess || hipSetDevice(s.device) != hipSuccess) continue;
    hipError_t e = hipEventSynchronize(s.hcopied[k]);
    if (e == hipSuccess && hc.staged[g] && __atomic_load_n(&s.pipe->ctl->timeout, __ATOMIC_ACQUIRE))
      e = hipErrorLaunchTimeOut;  // (a wave gave up waiting for a region: its chunks' verdicts are 0)
    if (e != hipSuccess && rc == AT2V_OK) rc = hip_code(e);
  }
  if (ctx->pipe_trace)
    std::fprintf(stderr, "[at2v pipe] n %zu: %.3f ms (host: wait %.3f, copy %.3f, enqueue %.3f ms)\n", hc.n,
                 std::chrono::duration<double>(std::chrono::steady_clock::now() - hc.t0).count() * 1e3,
                 ctx->tr_wait * 1e3, ctx->tr_copy * 1e3, ctx->tr_enq * 1e3);
  if (rc != AT2V_OK && ctx->cpu) {
    // AT2V_CTX_CPU_FALLBACK: the records are still in the caller's host buffers. Drain what the shards enqueued (no
    // verdict copy of this call may land after the CPU's words), then verify the whole batch on the CPU backend.
    for (Shard& s : ctx->shards) {
      if (hipSetDevice(s.device) != hipSuccess) continue;
      (void)hipStreamSynchronize(s.stream);
      if (s.pipe)
        for (hipStream_t st : {s.pipe->copy, s.pipe->comp[0], s.pipe->comp[1]}) (void)hipStreamSynchronize(st);
    }
    at2v::cpu_verify_batch(ctx->cpu, hc.pk, hc.sig, hc.msg, hc.msg_off, hc.n, (int)ctx->policy, hc.verdicts);
    ++ctx->cpu_batches;
    ++ctx->cpu_fallbacks;
    rc = AT2V_OK;
  }
  hc.rc = rc;
  hc.done = true;
}

// complete every host-buffer call still in flight (their results stay for at2v_verify_batch_wait)
void drain_host_calls(at2v_ctx* ctx) {
  int prev = 0;
  (void)hipGetDevice(&prev);
  for (uint64_t t = ctx->next_ticket > 2 ? ctx->next_ticket - 2 : 1; t < ctx->next_ticket; ++t)
    if (ctx->calls[t % 2].ticket == t) host_call_finish(ctx, (int)(t % 2));
  (void)hipSetDevice(prev);
}

int host_call_check(at2v_ctx* ctx, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, const uint32_t* msg_off,
                    size_t n, uint32_t* verdicts) {
  if (!ctx) return AT2V_E_INVALID;
  if (n == 0) return AT2V_OK;
  if (!pk || !sig || !msg_off || !verdicts || n >= (1u << 31)) return AT2V_E_INVALID;
  if (!msg && msg_off[n] != msg_off[0]) return AT2V_E_INVALID;
  if (!at2v::offsets_valid(msg_off, n)) return AT2V_E_INVALID;  // whole batch, before any device work
  return AT2V_OK;
}

}  // namespace

int at2v_verify_batch_submit(at2v_ctx* ctx, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg,
                             const uint32_t* msg_off, size_t n, uint32_t* verdicts, uint64_t* ticket) {
  if (!ticket) return AT2V_E_INVALID;
  *ticket = 0;
  const int chk = host_call_check(ctx, pk, sig, msg, msg_off, n, verdicts);
  if (chk != AT2V_OK) return chk;
  const uint64_t t = ctx->next_ticket++;
  const int k = (int)(t % 2);
  HostCall& hc = ctx->calls[k];
  int prev = 0;
  (void)hipGetDevice(&prev);
  host_call_finish(ctx, k);  // the call two tickets back: its slot's bitmaps and arenas are reused (its result is lost
                             // unless waited for; at most two calls are in flight)
  if (ctx->staged) drain_host_calls(ctx);  // (the staged form's ready word serves one call at a time)
  hc = HostCall{};
  hc.active = true;
  hc.ticket = t;
  hc.pk = pk;
  hc.sig = sig;
  hc.msg = msg;
  hc.msg_off = msg_off;
  hc.n = n;
  hc.verdicts = verdicts;
  *ticket = t;
  if (n == 0) {
    hc.done = true;
  } else if (ctx->shards.empty()) {  // CPU context: verified now
    at2v::cpu_verify_batch(ctx->cpu, pk, sig, msg, msg_off, n, (int)ctx->policy, verdicts);
    ++ctx->cpu_batches;
    hc.done = true;
  } else {
    host_call_issue(ctx, k);
  }
  (void)hipSetDevice(prev);
  return AT2V_OK;
}

int at2v_verify_batch_wait(at2v_ctx* ctx, uint64_t ticket) {
  if (!ctx || ticket == 0 || ticket >= ctx->next_ticket) return AT2V_E_INVALID;
  HostCall& hc = ctx->calls[ticket % 2];
  if (hc.ticket != ticket || !hc.active) return AT2V_E_INVALID;  // already waited for, or two or more calls back
  int prev = 0;
  (void)hipGetDevice(&prev);
  host_call_finish(ctx, (int)(ticket % 2));
  (void)hipSetDevice(prev);
  hc.active = false;
  return hc.rc;
}

int at2v_verify_batch(at2v_ctx* ctx, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg,
                      const uint32_t* msg_off, size_t n, uint32_t* verdicts) {
  const int chk = host_call_check(ctx, pk, sig, msg, msg_off, n, verdicts);
  if (chk != AT2V_OK || n == 0) return chk;
  if (ctx->shards.empty()) {  // CPU context
    at2v::cpu_verify_batch(ctx->cpu, pk, sig, msg, msg_off, n, (int)ctx->policy, verdicts);
    ++ctx->cpu_batches;
    return AT2V_OK;
  }
  int prev = 0;
  (void)hipGetDevice(&prev);
  drain_host_calls(ctx);
  HostCall& hc = ctx->calls[2];
  hc = HostCall{};
  hc.active = true;
  hc.pk = pk;
  hc.sig = sig;
  hc.msg = msg;
  hc.msg_off = msg_off;
  hc.n = n;
  hc.verdicts = verdicts;
  host_call_issue(ctx, 2);
  host_call_finish(ctx, 2);
  hc.active = false;
  (void)hipSetDevice(prev);
  return hc.rc;
}

int at2v_verify_batch_device(at2v_ctx* ctx, const uint8_t* d_pk, const uint8_t* d_sig, const uint8_t* d_msg,
                             size_t msg_bytes, const uint32_t* d_msg_off, size_t n, uint32_t* d_verdicts,
                             void* hip_stream) {
  if (!ctx) return AT2V_E_INVALID;
  if (n == 0) return AT2V_OK;
  if (!d_pk || !d_sig || !d_msg_off || !d_verdicts || n >= (1u << 31) || msg_bytes >= (1ull << 32))
    return AT2V_E_INVALID;
  if (ctx->shards.empty()) return AT2V_E_NODEVICE;
  if (!aligned(d_pk, 16) || !aligned(d_sig, 16) || !aligned(d_msg_off, 4) || !aligned(d_verdicts, 4))
    return AT2V_E_ALIGN;
  Shard& s = ctx->shards[0];
  int prev = 0;
  (void)hipGetDevice(&prev);
  hipError_t e = hipSetDevice(s.device);
  if (e == hipSuccess)
    e = launch_shard(ctx, s, d_pk, d_sig, d_msg, (uint32_t)msg_bytes, d_msg_off, (uint32_t)n, d_verdicts,
                     (hipStream_t)hip_stream);
  (void)hipSetDevice(prev);
  return hip_code(e);
}

// ---- RCCL: one rank per process ----

int at2v_comm_get_unique_id(uint8_t out[AT2V_UNIQUE_ID_BYTES]) {
  if (!out) return AT2V_E_INVALID;
  static_assert(AT2V_UNIQUE_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "unique id size");
  ncclUniqueId id;
  const ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) return AT2V_E_RCCL;
  std::memcpy(out, id.internal, AT2V_UNIQUE_ID_BYTES);
  return AT2V_OK;
}

int at2v_comm_init_rank(at2v_ctx* ctx, const uint8_t unique_id[AT2V_UNIQUE_ID_BYTES], int rank, int world) {
  if (ctx && ctx->shards.empty()) return AT2V_E_NODEVICE;
  if (!ctx || !unique_id || world < 1 || rank < 0 || rank >= world || ctx->comm || ctx->shards.size() != 1)
    return AT2V_E_INVALID;
  ncclUniqueId id;
  std::memcpy(id.internal, unique_id, AT2V_UNIQUE_ID_BYTES);
  int prev = 0;
  (void)hipGetDevice(&prev);
  int rc = hip_code(hipSetDevice(ctx->shards[0].device));
  // the failure-path buffers exist before the first collective, so a rank that fails later can still join it (the
  // status word itself is allocated by at2v_create, so the outcome all-reduce below can always be joined)
  if (rc == AT2V_OK) rc = hip_code(ctx->zeros.ensure(kGatherWindow * 4));
  if (rc == AT2V_OK) rc = hip_code(hipMemset(ctx->zeros.p, 0, ctx->zeros.cap));
  if (rc == AT2V_OK) rc = hip_code(ctx->window.ensure(kGatherWindow * 4 * (size_t)world));
  if (rc == AT2V_OK && !ctx->gather_done) {
    rc = hip_code(hipEventCreateWithFlags(&ctx->gather_done, hipEventDisableTiming));
    if (rc == AT2V_OK) rc = hip_code(hipEventRecord(ctx->gather_done, ctx->shards[0].stream));  // first wait: no-op
  }
  if (rc == AT2V_OK && at2v::test_env("AT2V_TEST_FAIL_COMM_SETUP")) rc = AT2V_E_HIP;  // test hook: a local set-up failure
  // collective: blocks until all `world` ranks have called it (a rank that failed above still joins, then reports)
  const int rn = nccl_code(ncclCommInitRank(&ctx->comm, world, id, rank));
  if (rn == AT2V_OK) {  // every rank that holds a communicator joins the outcome all-reduce, whatever failed locally
    // agree on the outcome: if any rank failed its local set-up, every rank drops the communicator, so no rank is left
    // with a peer that will never join its collectives
    int got = 1;
    hipStream_t st = ctx->shards[0].stream;
    hipError_t es = hipMemsetD32Async((hipDeviceptr_t)ctx->status.p, rc != AT2V_OK, 1, st);
    const ncclResult_t ra = ncclAllReduce(ctx->status.p, ctx->status.p, 1, ncclInt32, ncclMax, ctx->comm, st);
    if (es == hipSuccess) es = hipMemcpyAsync(&got, ctx->status.p, 4, hipMemcpyDeviceToHost, st);
    if (es == hipSuccess) es = hipStreamSynchronize(st);
    if (rc == AT2V_OK && (ra != ncclSuccess || es != hipSuccess)) rc = ra != ncclSuccess ? AT2V_E_RCCL : hip_code(es);
    if (rc == AT2V_OK && got) rc = AT2V_E_PEER;
  }
  if (rc == AT2V_OK) rc = rn;
  if (rc == AT2V_OK) {
    ctx->rank = rank;
    ctx->world = world;
  } else {
    if (ctx->comm) (void)ncclCommDestroy(ctx->comm);
    ctx->comm = nullptr;
  }
  (void)hipSetDevice(prev);
  return rc;
}

int at2v_verify_shard_gather_device(at2v_ctx* ctx, const uint8_t* d_pk, const uint8_t* d_sig, const uint8_t* d_msg,
                                    size_t msg_bytes, const uint32_t* d_msg_off, size_t n_local,
                                    size_t words_per_rank, uint32_t* d_bitmap, void* hip_stream) {
  // Without a communicator, a bitmap or a word count every rank agrees on, the collective cannot be joined at all:
  // these are contract violations that every rank of a correct caller makes alike.
  if (!ctx || !ctx->comm || !d_bitmap || words_per_rank == 0 || words_per_rank >= (1ull << 26))
    return AT2V_E_INVALID;
  if (!aligned(d_bitmap, 4)) return AT2V_E_ALIGN;
  // Anything else is this rank's own problem: it still joins the all-gather with a zero slice (gather_shard).
  int local = AT2V_OK;
  if (n_local > 32 * words_per_rank || (n_local && (!d_pk || !d_sig || !d_msg_off)) || msg_bytes >= (1ull << 32))
    local = AT2V_E_INVALID;
  else if (n_local && (!aligned(d_pk, 16) || !aligned(d_sig, 16) || !aligned(d_msg_off, 4)))
    local = AT2V_E_ALIGN;
  Shard& s = ctx->shards[0];
  int prev = 0;
  (void)hipGetDevice(&prev);
  const hipError_t e = hipSetDevice(s.device);
  if (e != hipSuccess && local == AT2V_OK) local = hip_code(e);
  const int rc = gather_shard(ctx, s, local, d_pk, d_sig, d_msg, msg_bytes, d_msg_off, n_local, words_per_rank,
                              d_bitmap, (hipStream_t)hip_stream);
  (void)hipSetDevice(prev);
  return rc;
}

int at2v_verify_batch_sharded(at2v_ctx* ctx, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg,
                              const uint32_t* msg_off, size_t n, uint32_t* verdicts) {
  // Argument checks on the WHOLE node batch, which every rank receives identically: either every rank returns here
  // or none does (a bad offset seen by one rank only used to leave the others inside the all-gather).
  if (!ctx || !ctx->comm || n >= (1u << 31)) return AT2V_E_INVALID;
  if (n && (!pk || !sig || !msg_off || !verdicts || (!msg && msg_off[n] != msg_off[0]))) return AT2V_E_INVALID;
  if (n && !at2v::offsets_valid(msg_off, n)) return AT2V_E_INVALID;
  drain_host_calls(ctx);  // (they share the shard's pipe)
  Shard& s = ctx->shards[0];
  const size_t wpr = at2v::shard_words_per_rank(n, ctx->world);
  const at2v::Range r = at2v::rank_range(n, ctx->world, ctx->rank);
  const size_t a = r.lo, m = r.size();
  int prev = 0;
  (void)hipGetDevice(&prev);
  hipError_t e = hipSetDevice(s.device);
  // Local steps: this rank's range through the chunked pipeline (HostPipe) into its wpr words, pad words zeroed. A failure
  // here is this rank's alone: it still joins every collective below, sending zero words (fail closed), and every rank
  // learns of it. The collectives run on the pipe's copy stream (the context's own stream if the pipe could not be made),
  // behind the chunks' launches; the sender cache's builds run on the context's stream and do not delay them.
  if (e == hipSuccess) e = s.verdict.ensure(wpr * 4);
  if (e == hipSuccess) e = ensure_pipe(s, ctx->pipe_streams);
  hipStream_t st = s.pipe ? s.pipe->copy : s.stream;
  const size_t used = (m + 31) / 32;  // words the chunks' launches write (each zeroes its own first)
  if (e == hipSuccess && used < wpr)
    e = hipMemsetAsync((uint32_t*)s.verdict.p + used, 0, (wpr - used) * 4, st);  // pad words (an empty rank: all)
  if (e == hipSuccess && m) e = begin_arena(ctx, s, m, (size_t)(msg_off[a + m] - msg_off[a]));
  if (e == hipSuccess && m) {
    at2v::CpuPool* copier = copy_pool(ctx);
    ChunkPlan cp;
    cp.init(m, ctx);
    while (e == hipSuccess && !cp.done()) {
      const size_t at = cp.pos, c = cp.take();
      e = issue_chunk(ctx, s, copier, pk, sig, msg, msg_off, a + at, c, (uint32_t*)s.verdict.p + at / 32,
                      m > ctx->pair_max, at == 0);
    }
    const hipError_t ef = flush_chunk(ctx, s);  // the last chunk
    if (e == hipSuccess) e = ef;
    for (int j = 0; j < 2 && e == hipSuccess; ++j) e = hipStreamWaitEvent(st, s.pipe->comp_done[j], 0);
  }
  int rc = hip_code(e);
  // The all-gather runs in rounds of at most kGatherWindow words per rank through buffers allocated at
  // at2v_comm_init_rank, so no allocation stands between a rank and the collectives: every rank issues the same
  // ceil(wpr / window) all-gathers whatever happened locally.
  if (ctx->gather_done) (void)hipStreamWaitEvent(st, ctx->gather_done, 0);
  const size_t W = kGatherWindow;
  for (size_t j0 = 0; j0 < wpr; j0 += W) {
    const size_t cnt = std::min(W, wpr - j0);
    const void* send = rc == AT2V_OK ? (const void*)((const uint32_t*)s.verdict.p + j0) : ctx->zeros.p;
    const ncclResult_t rr = ncclAllGather(send, ctx->window.p, cnt, ncclUint32, ctx->comm, st);
    ++ctx->gathers;
    if (rr != ncclSuccess && rc == AT2V_OK) rc = AT2V_E_RCCL;
    // rank q's words [j0, j0 + cnt) are at window word q * cnt; its real words go to word lo_q/32 + j0 of verdicts
    for (int q = 0; q < ctx->world && n; ++q) {
      const at2v::WordCopy wc = at2v::rank_words(n, ctx->world, q);
      if (wc.words <= j0) continue;
      const size_t k = std::min(cnt, wc.words - j0);
      const hipError_t ec = hipMemcpyAsync(verdicts + wc.dst_word + j0, (const uint32_t*)ctx->window.p + (size_t)q * cnt,
                                           k * 4, hipMemcpyDeviceToHost, st);
      if (ec != hipSuccess && rc == AT2V_OK) rc = hip_code(ec);
    }
    const hipError_t es = hipStreamSynchronize(st);  // the window is reused by the next round
    if (es != hipSuccess && rc == AT2V_OK) rc = hip_code(es);
  }
  if (ctx->gather_done) (void)hipEventRecord(ctx->gather_done, st);
  // Every rank learns whether any rank failed: a peer's failure turns this rank's success into AT2V_E_PEER, so no
  // rank hands a bitmap with a zeroed (fail-closed) slice to its apply step as if it were complete.
  int any = rc != AT2V_OK;
  hipError_t es = hipMemsetD32Async((hipDeviceptr_t)ctx->status.p, any, 1, st);
  const ncclResult_t ra = ncclAllReduce(ctx->status.p, ctx->status.p, 1, ncclInt32, ncclMax, ctx->comm, st);
  int got = 1;
  if (es == hipSuccess) es = hipMemcpyAsync(&got, ctx->status.p, 4, hipMemcpyDeviceToHost, st);
  if (es == hipSuccess) es = hipStreamSynchronize(st);
  if (rc == AT2V_OK && ra != ncclSuccess) rc = AT2V_E_RCCL;
  if (rc == AT2V_OK && es != hipSuccess) rc = hip_code(es);
  if (rc == AT2V_OK && got) rc = AT2V_E_PEER;
  (void)hipSetDevice(prev);
  return rc;
}

const char* at2v_strerror(int code) {
  switch (code) {
    case AT2V_OK: return "ok";
    case AT2V_E_INVALID: return "invalid argument";
    case AT2V_E_NODEVICE: return "no usable gfx950 device (or a device entry point on a CPU context)";
    case AT2V_E_HIP: return "HIP runtime error";
    case AT2V_E_OOM: return "out of memory";
    case AT2V_E_ALIGN: return "misaligned device pointer";
    case AT2V_E_RCCL: return "RCCL error";
    case AT2V_E_PEER: return "another rank failed this collective batch (its records are verdict 0)";
    default: return "unknown error";
  }
}

int at2v_gen_records_device(at2v_ctx* ctx, uint64_t cfg_seed, uint64_t first, size_t n, uint32_t msg_len,
                            uint8_t* d_pk, uint8_t* d_sig, uint8_t* d_msg, uint32_t* d_msg_off, void* hip_stream) {
  return at2v_gen_records_senders_device(ctx, cfg_seed, first, n, msg_len, 0, d_pk, d_sig, d_msg, d_msg_off,
                                         hip_stream);
}

static int gen_records(at2v_ctx* ctx, uint64_t cfg_seed, uint64_t first, size_t n, uint32_t msg_len, uint64_t senders,
                       const uint64_t* d_keys, uint8_t* d_pk, uint8_t* d_sig, uint8_t* d_msg, uint32_t* d_msg_off,
                       void* hip_stream) {
  if (!ctx) return AT2V_E_INVALID;
  if (n == 0) return AT2V_OK;
  if (!d_pk || !d_sig || (!d_msg && msg_len) || n >= (1u << 31) || (uint64_t)n * msg_len >= (1ull << 32))
    return AT2V_E_INVALID;
  if (ctx->shards.empty()) return AT2V_E_NODEVICE;
  if (!aligned(d_pk, 4) || !aligned(d_sig, 4) || (d_msg_off && !aligned(d_msg_off, 4)) || !aligned(d_keys, 8))
    return AT2V_E_ALIGN;
  Shard& s = ctx->shards[0];
  int prev = 0;
  (void)hipGetDevice(&prev);
  hipError_t e = hipSetDevice(s.device);
  if (e == hipSuccess)
    e = at2v::launch_gen(cfg_seed, first, (uint32_t)n, msg_len, senders, d_keys, d_pk, d_sig, d_msg, d_msg_off,
                         (hipStream_t)hip_stream);
  (void)hipSetDevice(prev);
  return hip_code(e);
}

int at2v_gen_records_senders_device(at2v_ctx* ctx, uint64_t cfg_seed, uint64_t first, size_t n, uint32_t msg_len,
                                    uint64_t senders, uint8_t* d_pk, uint8_t* d_sig, uint8_t* d_msg,
                                    uint32_t* d_msg_off, void* hip_stream) {
  return gen_records(ctx, cfg_seed, first, n, msg_len, senders, nullptr, d_pk, d_sig, d_msg, d_msg_off, hip_stream);
}

int at2v_gen_records_keys_device(at2v_ctx* ctx, uint64_t cfg_seed, uint64_t first, size_t n, uint32_t msg_len,
                                 const uint64_t* d_keys, uint8_t* d_pk, uint8_t* d_sig, uint8_t* d_msg,
                                 uint32_t* d_msg_off, void* hip_stream) {
  if (n && !d_keys) return AT2V_E_INVALID;
  return gen_records(ctx, cfg_seed, first, n, msg_len, 0, d_keys, d_pk, d_sig, d_msg, d_msg_off, hip_stream);
}

int at2v_sign_batch(at2v_ctx* ctx, const uint8_t* seeds, const uint8_t* msg, const uint32_t* msg_off, size_t n,
                    uint8_t* pk_out, uint8_t* sig_out) {
  if (!ctx) return AT2V_E_INVALID;
  if (n == 0) return AT2V_OK;
  if (!seeds || !msg_off || !pk_out || !sig_out || n >= (1u << 31)) return AT2V_E_INVALID;
  if (ctx->shards.empty()) return AT2V_E_NODEVICE;  // (signing is the client's side, not the verify path)
  Shard& s = ctx->shards[0];
  const uint32_t mb0 = msg_off[0], mb1 = msg_off[n];
  if (mb1 < mb0 || (!msg && mb1 != mb0)) return AT2V_E_INVALID;
  const size_t mbytes = mb1 - mb0;
  std::vector<uint32_t> offs(n + 1);
  for (size_t i = 0; i <= n; ++i) {
    offs[i] = msg_off[i] - mb0;
    if (i && offs[i] < offs[i - 1]) return AT2V_E_INVALID;
  }
  int prev = 0;
  (void)hipGetDevice(&prev);
  DevBuf dseed, dmsg, doff, dpk, dsig;
  hipError_t e = hipSetDevice(s.device);
  if (e == hipSuccess) e = dseed.ensure(n * 32);
  if (e == hipSuccess) e = dmsg.ensure(mbytes + 16);
  if (e == hipSuccess) e = doff.ensure((n + 1) * 4);
  if (e == hipSuccess) e = dpk.ensure(n * 32);
  if (e == hipSuccess) e = dsig.ensure(n * 64);
  if (e == hipSuccess) e = hipMemcpyAsync(dseed.p, seeds, n * 32, hipMemcpyHostToDevice, s.stream);
  if (e == hipSuccess && mbytes) e = hipMemcpyAsync(dmsg.p, msg + mb0, mbytes, hipMemcpyHostToDevice, s.stream);
  if (e == hipSuccess) e = hipMemcpyAsync(doff.p, offs.data(), (n + 1) * 4, hipMemcpyHostToDevice, s.stream);
  if (e == hipSuccess)
    e = at2v::launch_sign((const uint8_t*)dseed.p, (const uint8_t*)dmsg.p, (uint32_t)mbytes, (const uint32_t*)doff.p,
                          (uint32_t)n, (uint8_t*)dpk.p, (uint8_t*)dsig.p, s.stream);
  if (e == hipSuccess) e = hipMemcpyAsync(pk_out, dpk.p, n * 32, hipMemcpyDeviceToHost, s.stream);
  if (e == hipSuccess) e = hipMemcpyAsync(sig_out, dsig.p, n * 64, hipMemcpyDeviceToHost, s.stream);
  if (e == hipSuccess) e = hipStreamSynchronize(s.stream);
  dseed.release();
  dmsg.release();
  doff.release();
  dpk.release();
  dsig.release();
  (void)hipSetDevice(prev);
  return hip_code(e);
}

int at2v_decode_points(at2v_ctx* ctx, const uint8_t* pts, size_t n, uint32_t* valid_words) {
  if (!ctx) return AT2V_E_INVALID;
  if (n == 0) return AT2V_OK;
  if (!pts || !valid_words || n >= (1u << 31)) return AT2V_E_INVALID;
  if (ctx->shards.empty()) {  // CPU context: the kernels' decode routine on the host
    at2v::cpu_decode_points(ctx->cpu, pts, n, valid_words);
    return AT2V_OK;
  }
  Shard& s = ctx->shards[0];
  int prev = 0;
  (void)hipGetDevice(&prev);
  const size_t words = (n + 31) / 32;
  hipError_t e = hipSetDevice(s.device);
  if (e == hipSuccess) e = s.pk.ensure(n * 32);
  if (e == hipSuccess) e = s.verdict.ensure(words * 4);
  if (e == hipSuccess) e = hipMemcpyAsync(s.pk.p, pts, n * 32, hipMemcpyHostToDevice, s.stream);
  if (e == hipSuccess) e = at2v::launch_decode((const uint8_t*)s.pk.p, (uint32_t)n, (uint32_t*)s.verdict.p, s.stream);
  if (e == hipSuccess) e = hipMemcpyAsync(valid_words, s.verdict.p, words * 4, hipMemcpyDeviceToHost, s.stream);
  if (e == hipSuccess) e = hipStreamSynchronize(s.stream);
  (void)hipSetDevice(prev);
  return hip_code(e);
}

int at2v_get_info(at2v_ctx* ctx, at2v_info* out) {
  if (!ctx || !out) return AT2V_E_INVALID;
  std::memset(out, 0, sizeof *out);
  out->cpu_threads = at2v::cpu_pool_threads(ctx->cpu);
  out->cpu_batches = ctx->cpu_batches;
  out->cpu_fallbacks = ctx->cpu_fallbacks;
  out->experiments = library_experiments();
  out->host_chunks = ctx->host_chunks;
  if (ctx->shards.empty()) return AT2V_OK;  // CPU context: no device geometry
  const Shard& s = ctx->shards[0];
  out->num_gpus = (int)ctx->shards.size();
  out->grid_blocks = s.grid;
  out->block_threads = at2v::block_threads();
  out->waves_per_cu = s.blocks_per_cu * at2v::block_threads() / 64;
  out->cus = s.cus;
  out->vgprs = s.vgprs;
  out->rank = ctx->rank;
  out->world = ctx->comm ? ctx->world : 0;
  out->gathers = ctx->gathers;
  for (const Shard& sh : ctx->shards) {
    // sender-cache counters, summed over devices. Waits for the context's cache work only (its build stream, which
    // follows every cached launch): builds of earlier launches are done and their keys usable when this returns.
    if (!sh.cache) continue;
    std::vector<unsigned long long> w((size_t)at2v::cache_ctl_words());
    int prev = 0;
    (void)hipGetDevice(&prev);
    if (hipSetDevice(sh.device) == hipSuccess && hipStreamSynchronize(sh.cache->build) == hipSuccess &&
        hipMemcpyAsync(w.data(), sh.cache->ctl.p, w.size() * 8, hipMemcpyDeviceToHost, sh.cache->build) == hipSuccess &&
        hipStreamSynchronize(sh.cache->build) == hipSuccess) {
      const uint64_t fc = w[at2v::kCtlFreeCount], fh = w[at2v::kCtlFreeHead];
      const uint64_t cap = sh.cache->args.capacity;
      out->cache_entries += (cap - std::min(fc, cap)) + std::min(fh, fc);  // keys holding a payload
      out->cache_chunks += w[at2v::kCtlChunks];
      out->cache_chunk_hits += w[at2v::kCtlChunkHits];
      out->cache_claims += w[at2v::kCtlClaimed];
      out->cache_evicted += w[at2v::kCtlEvicted];
      out->cache_compactions += w[at2v::kCtlCompactions];
      out->cache_sightings += w[at2v::kCtlSighted];
      out->cache_built += w[at2v::kCtlBuilt];
      out->cache_record_hits += w[at2v::kCtlRecHits];
      int khz = 0;  // device wall clock (wall_clock64) in kHz
      if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, sh.device) == hipSuccess && khz > 0)
        out->cache_build_us += w[at2v::kCtlBuildTicks] * 1000ull / (uint64_t)khz;
      out->cache_capacity += cap;
    }
    (void)hipSetDevice(prev);
  }
  return AT2V_OK;
}

int at2v_abi_version(void) { return AT2V_ABI_VERSION; }

}  // extern "C"
