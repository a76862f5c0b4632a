/*
 * at2v.h — C ABI of the MI355X batch Ed25519 verifier for the at2-node server hot path.
 *
 * Drop-in boundary. In the reference (Rust, /root/reference) every client
 * signature is checked one at a time by the external `drop::crypto::sign` verify that
 * sieve/murmur call per payload:
 *   - payloads enter at   src/bin/server/rpc.rs:275-284  (broadcast(sieve::Payload::new(sender, seq, thin, sig)))
 *   - verified batches at src/bin/server/rpc.rs:156-173  (deliver() -> batch -> apply heap)
 *   - signed message M  = bincode(ThinTransaction)  src/lib.rs:14-22, signed at src/client.rs:77-78
 *   - A decoded at rpc.rs:269, signature decoded at rpc.rs:281
 * This library replaces that per-signature call with a batch call whose verdicts are identical
 * (ed25519-dalek 1.x `PublicKey::verify` semantics: cofactorless, s < l, dalek point decoding,
 * byte comparison of the canonical R encoding). The Rust binding a maintainer
 * adds to the reference (extern "C" block + build.rs link line) is in INTEGRATION.md.
 *
 * All functions are noexcept; no C++ exception or HIP error escapes as anything but a negative code.
 */
#ifndef AT2V_H
#define AT2V_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI version of this header. Every struct passed by pointer is copied whole, so adding a field is an ABI break:
 * version 7 appended at2v_info.experiments / host_chunks (and the AT2V_EXPERIMENT_* bits) and added
 * at2v_verify_batch_submit / _wait; version 6 appended at2v_opts.cpu_threads / flags (num_gpus = 0 now means the CPU batch backend, no device),
 * at2v_info.cpu_threads / cpu_batches / cpu_fallbacks / cache_sightings / cache_built / cache_build_us /
 * cache_record_hits,
 * at2v_gen_records_keys_device, at2v_queue_opts.cpu_threads (with the
 * AT2V_QUEUE_CPU / AT2V_QUEUE_CPU_FALLBACK flags) and at2v_queue_stats.cpu_fallbacks; version 5 appended at2v_queue_opts.sender_cache and at2v_info.cache_capacity / cache_claims / cache_evicted /
 * cache_compactions (the sender cache replaces entries instead of restarting empty); version 4 appended
 * at2v_opts.sender_comb and the AT2V_QUEUE_SENDER_COMB queue flag; version 3 appended at2v_opts.sender_cache, at2v_info.gathers / cache_* and the AT2V_E_PEER code (version 2 appended
 * at2v_opts.small_batch_max and at2v_queue_opts.flags). A binding checks at2v_abi_version() == AT2V_ABI_VERSION
 * before passing any struct (the Python and Rust bindings in this repo refuse a mismatching library). */
#define AT2V_ABI_VERSION 7
int at2v_abi_version(void);

typedef struct at2v_ctx at2v_ctx; /* opaque: device(s), streams, scratch, staging buffers, and the RCCL
                                     communicator once at2v_comm_init_rank has attached one */

typedef enum {
  AT2V_POLICY_DALEK_V1 = 0,         /* ed25519-dalek 1.x PublicKey::verify (the reference; default) */
  AT2V_POLICY_LIBSODIUM_1_0_18 = 1  /* + libsodium 1.0.18 pre-rejects: A non-canonical / small order, R small order */
} at2v_policy;

typedef struct {
  int device;         /* first HIP device ordinal (default 0) */
  int num_gpus;       /* devices device..device+num_gpus-1 share each host batch by index range. 0 = the CPU batch
                         backend: no device is touched; at2v_verify_batch runs the kernels' own verify routine on
                         cpu_threads host threads (what SystemManager::run(.., num_cpus::get()) did, rpc.rs:124-125) */
  at2v_policy policy; /* verdict semantics */
  uint32_t small_batch_max; /* launches of at most this many records run the low-latency kernel (two lanes per
                               record, one wave per SIMD); 0 = 32768; AT2V_SMALL_BATCH_OFF = never */
  uint32_t sender_cache;    /* per-sender A cache (AT2 senders repeat: accounts/account.rs:36-43): capacity in distinct
                               public keys, 0 = off. A record whose sender A is cached skips decoding A and building
                               its [j]A table; the verdict is unchanged (the cache holds only values derived from the
                               32 bytes of A, and every hit is confirmed by comparing those bytes). A key seen for the
                               first time is verified without the cache; its entry is built on the context's build
                               stream after that launch and serves later launches. When the capacity is reached, the
                               least recently used entries (by launch) are replaced; up to 3/4 of the capacity stays. */
  uint32_t sender_comb;     /* with sender_cache: 1 = every cached key also gets a comb of -A ([j 2^(10i)](-A), 1.7 MB
                               per key, sender_cache x 1.7 MB per device, plus combs of B of 67 MB and 872 MB per context;
                               AT2V_CTX_BCOMB_WIDE widens the second), and a record whose sender is cached is verified by
                               39 table additions (37 with the wide comb of B) and one
                               inversion instead of the doubling ladder (~3x fewer multiplications; launches of any size,
                               small batches included). Same verdicts. 0 = off. */
  uint32_t cpu_threads;     /* host threads of the CPU backend (num_gpus = 0, or AT2V_CTX_CPU_FALLBACK): 0 = every CPU
                               this process may use (affinity mask, capped by a cgroup CPU quota) */
  uint32_t flags;           /* AT2V_CTX_* below */
} at2v_opts;
/* A GPU context that hits a device error inside at2v_verify_batch (host buffers: the records are still on the host)
 * verifies that batch again on the CPU backend and returns AT2V_OK with identical verdicts; at2v_info.cpu_fallbacks counts
 * it. Device-buffer entry points cannot fall back (their records live on the failed device) and return the error. */
#define AT2V_CTX_CPU_FALLBACK 1u
/* Sender cache admission: by default a key gets a cache payload (a [j]A table, or a 1.7 MB comb) only when it is seen
 * again in a later launch, or when one wave of a launch holds two or more of its records, so one-shot senders cost a
 * sighting (one 8-byte store) instead of a build. This flag admits every key at its first sighting (round-4 behaviour). */
#define AT2V_CTX_ADMIT_FIRST 2u
/* With sender_comb: the throughput kernel's cached records take [s]B from a comb of B with 24-bit windows (11 positions,
 * 11.8 GB of HBM per device) instead of the default 20-bit one (13 positions, 872 MB): two table additions fewer per
 * record (37 instead of 39), +3% on repeating senders. Opt-in for its memory and its 0.75 s of table build at context
 * creation; small-batch latency is unchanged with it. */
#define AT2V_CTX_BCOMB_WIDE 4u
#define AT2V_SMALL_BATCH_DEFAULT 32768u
#define AT2V_SMALL_BATCH_OFF 0xffffffffu

enum {
  AT2V_OK = 0,
  AT2V_E_INVALID = -1,  /* bad argument (NULL pointer, n too large, ...) */
  AT2V_E_NODEVICE = -2, /* no usable gfx950 device / library built without the HIP kernels */
  AT2V_E_HIP = -3,      /* HIP runtime error */
  AT2V_E_OOM = -4,      /* device or host allocation failed */
  AT2V_E_ALIGN = -5,    /* device pointer not 16-byte aligned (pk, sig) or 4-byte aligned (offsets, verdicts) */
  AT2V_E_RCCL = -6,     /* RCCL communicator / collective failure (at2v_comm_init_rank, the verdict all-gather) */
  AT2V_E_PEER = -7      /* at2v_verify_batch_sharded / at2v_comm_init_rank: this rank succeeded but another rank of the
                           communicator failed; that rank's records are verdict 0 (fail closed), discard the batch */
};

/* Timing-only experiment switches a library may have been compiled with (AT2V_EXP_* build macros; each makes some
 * verdicts WRONG). at2v_create fails with AT2V_E_INVALID on such a build unless the environment variable
 * AT2V_ALLOW_EXPERIMENT is "1", and at2v_info.experiments reports the bits. A shipped build has none. */
#define AT2V_EXPERIMENT_TAB128 1u        /* 128-byte [j]A table entries, the last 8 words dropped */
#define AT2V_EXPERIMENT_COMB_HOT 2u      /* every A-comb entry read is the same cache line */
#define AT2V_EXPERIMENT_SLOT_WAVES 4u    /* waves share per-lane table slots */
#define AT2V_EXPERIMENT_CONST_MSG 8u     /* message words from registers */
#define AT2V_EXPERIMENT_BCOMB_NOBUILD 16u /* the hit-list kernel's comb of B left unwritten */
#define AT2V_EXPERIMENT_COMB3 32u        /* hit-list comb kernel at three waves per SIMD, its two LDS stages aliased */

/* Create / destroy a context. opts may be NULL (device 0, one GPU, DALEK_V1). Replaces nothing in the
 * reference directly: it owns what drop's SystemManager::run(.., num_cpus::get()) workers did
 * implicitly (rpc.rs:124-125). A context is not thread-safe: one thread at a time. A device has two scratch sets that
 * its verify launches take in turn, whatever streams they are given: a launch waits (on the device) for the launch that
 * last used its set, so launches on two streams overlap by up to one launch and launches on one stream are ordered. */
int at2v_create(const at2v_opts* opts, at2v_ctx** out);
void at2v_destroy(at2v_ctx* ctx);

/* Batch verify, host buffers. Replaces N calls of drop::crypto::sign verify (per payload, inside
 * sieve/murmur) for the payloads a node receives (rpc.rs:275-284 → rpc.rs:156).
 *   pk       n x 32 bytes   (sender public key A = bincode-decoded SendAssetRequest.sender, at2.proto:11)
 *   sig      n x 64 bytes   (R || S = SendAssetRequest.signature, at2.proto:15)
 *   msg      concatenated messages; message i = msg[msg_off[i] .. msg_off[i+1]) (M = bincode(ThinTransaction))
 *   msg_off  n + 1 offsets, non-decreasing, msg_off[0] may be > 0
 *   verdicts ceil(n/32) words out; bit (i % 32) of word (i / 32) = 1 iff record i is valid. Pad bits are 0.
 * Malformed records (undecodable A, s >= l, wrong equation, ...) are verdict 0, never an error.
 * The library does not retain any pointer after return. n may be 0. n < 2^31. */
int at2v_verify_batch(at2v_ctx* ctx, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg,
                      const uint32_t* msg_off, size_t n, uint32_t* verdicts);

/* The same call in two halves, so that a caller can stage its next batch while the device verifies this one (the
 * synchronous call leaves the device idle while it copies its first chunk and after it returns).
 * at2v_verify_batch_submit validates the batch, copies it to the device and enqueues its launches and its verdict
 * download, then returns a ticket (> 0). The caller's arrays, verdicts included, must stay valid and unchanged until
 * at2v_verify_batch_wait(ctx, ticket) has returned; only then are the verdict words final. At most two calls are in
 * flight per context: a submit completes the call two tickets back first (its verdicts land; its result code is lost
 * unless it was waited for). Waiting returns that call's result: AT2V_OK, or the error at2v_verify_batch would have
 * returned (with AT2V_CTX_CPU_FALLBACK the batch is re-verified on the CPU inside the wait). A ticket is waited for
 * once; an unknown, repeated or too old ticket gives AT2V_E_INVALID. at2v_verify_batch and at2v_verify_batch_sharded
 * complete the calls in flight first (their results stay for their waits). Validation errors are returned by the
 * submit (no ticket). */
int at2v_verify_batch_submit(at2v_ctx* ctx, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg,
                             const uint32_t* msg_off, size_t n, uint32_t* verdicts, uint64_t* ticket);
int at2v_verify_batch_wait(at2v_ctx* ctx, uint64_t ticket);

/* Batch verify on device-resident buffers of ctx's first device (AT2V_E_NODEVICE on a CPU context), asynchronously on
 * `hip_stream`
 * (a hipStream_t; NULL = the null stream). Same layout as at2v_verify_batch; msg_bytes = size of the
 * msg buffer in bytes (>= msg_off[n]); d_pk/d_sig 16-byte aligned, d_msg_off/d_verdicts 4-byte aligned.
 * Returns after the launch; results are valid once the stream reaches this point. The ceil(n/32) verdict
 * words are zeroed on the stream before the kernel runs. The launch first waits (on the device, not the
 * host) for the launch that last used the scratch set it takes (a device has two, used in turn), which may be on
 * another stream: launches on two streams overlap, launches on one stream are ordered by it. */
int at2v_verify_batch_device(at2v_ctx* ctx, const uint8_t* d_pk, const uint8_t* d_sig, const uint8_t* d_msg,
                             size_t msg_bytes, const uint32_t* d_msg_off, size_t n, uint32_t* d_verdicts,
                             void* hip_stream);

/* One signature on the CPU, synchronous: 1 = valid, 0 = invalid, < 0 = error. The drop-in for the
 * per-signature `Signature::verify(&message, &public_key)` that drop exposes and sieve/murmur call per payload
 * ("CPU, 1/0"), for callers that verify one payload at a time, e.g. the A/sig decode at
 * rpc.rs:265-281. DALEK_V1 semantics: the throughput kernel's own verify routine (csrc/at2v_verify_fu.h)
 * compiled for the host; needs no GPU, no context and no lock; reentrant (the first call of a process builds the
 * fixed-base tables, ~30 ms). A CPU context (num_gpus = 0) and the AT2V_CTX_CPU_FALLBACK path run the same routine
 * over a thread pool. */
int at2v_verify_one(const uint8_t pk[32], const uint8_t sig[64], const uint8_t* msg, size_t len);
/* Same, with an explicit policy (AT2V_POLICY_*). */
int at2v_verify_one_policy(const uint8_t pk[32], const uint8_t sig[64], const uint8_t* msg, size_t len, int policy);

const char* at2v_strerror(int code);

/* ---- signing side (client, src/client.rs:77-78), used to synthesise inputs on the GPU ---- */

/* Deterministic synthetic records (SURVEY §8(d) generator), written on ctx's first device:
 *   seed_i = SHA-512("at2v/seed" || u64le(cfg_seed) || u64le(i))[0:32]
 *   M_i    = SHA-512("at2v/msg" || u64le(cfg_seed) || u64le(i) || u64le(ctr)) stream, msg_len bytes
 *   (A_i, R_i || S_i) = RFC 8032 keygen/sign of M_i under seed_i
 * for i = first .. first+n-1. d_msg receives n*msg_len bytes, d_msg_off (may be NULL) n+1 offsets
 * i*msg_len. Asynchronous on hip_stream. */
int at2v_gen_records_device(at2v_ctx* ctx, uint64_t cfg_seed, uint64_t first, size_t n, uint32_t msg_len,
                            uint8_t* d_pk, uint8_t* d_sig, uint8_t* d_msg, uint32_t* d_msg_off, void* hip_stream);

/* The same with repeating senders (AT2 traffic: accounts/account.rs:36-43): record i is signed by the key of seed index
 * (first + i) % senders, its message is still M_i. senders = 0: distinct keys (= at2v_gen_records_device). */
int at2v_gen_records_senders_device(at2v_ctx* ctx, uint64_t cfg_seed, uint64_t first, size_t n, uint32_t msg_len,
                                    uint64_t senders, uint8_t* d_pk, uint8_t* d_sig, uint8_t* d_msg,
                                    uint32_t* d_msg_off, void* hip_stream);

/* The same with an explicit key per record: record i is signed by the key of seed index d_keys[i] (n u64 on the device,
 * 8-byte aligned), its message is still M_(first+i). For traffic with a chosen sender distribution (bench: Zipf). */
int at2v_gen_records_keys_device(at2v_ctx* ctx, uint64_t cfg_seed, uint64_t first, size_t n, uint32_t msg_len,
                                 const uint64_t* d_keys, uint8_t* d_pk, uint8_t* d_sig, uint8_t* d_msg,
                                 uint32_t* d_msg_off, void* hip_stream);

/* RFC 8032 signing of host messages under 32-byte seeds (host buffers, synchronous). pk_out n x 32,
 * sig_out n x 64. The GPU counterpart of KeyPair::sign (drop), used by tests and the bench generator. */
int at2v_sign_batch(at2v_ctx* ctx, const uint8_t* seeds, const uint8_t* msg, const uint32_t* msg_off, size_t n,
                    uint8_t* pk_out, uint8_t* sig_out);

/* Introspection for benches: kernel geometry actually used by the last verify launch. */
typedef struct {
  int num_gpus;        /* 0: a CPU-backend context (the geometry fields below are then 0) */
  int grid_blocks;     /* per device */
  int block_threads;
  int waves_per_cu;    /* resident waves per CU admitted by the kernel's register/LDS use */
  int cus;             /* compute units of the first device */
  int vgprs;           /* VGPRs per lane of the verify kernel (from the code object) */
  int rank;            /* at2v_comm_init_rank: this context's rank, else 0 */
  int world;           /* at2v_comm_init_rank: ranks in the communicator, else 0 */
  uint64_t gathers;    /* verdict all-gathers this context has issued (failure paths included) */
  uint64_t cache_entries;    /* at2v_opts.sender_cache: distinct senders now cached (all devices) */
  uint64_t cache_chunks;     /* 64-record chunks verified with the cache on */
  uint64_t cache_chunk_hits; /* ... of which every record's A came from the cache (A decode and [j]A skipped) */
  uint64_t cache_capacity;   /* keys the cache can hold (all devices) */
  uint64_t cache_claims;     /* keys claimed (first seen, or seen again after being replaced) */
  uint64_t cache_evicted;    /* entries replaced to make room */
  uint64_t cache_compactions;/* replacement passes */
  uint64_t cpu_threads;      /* threads of the context's CPU backend (0: none) */
  uint64_t cpu_batches;      /* batches verified on the CPU backend (a CPU context's batches, and fallbacks) */
  uint64_t cpu_fallbacks;    /* ... of which a GPU context re-ran after a device error (AT2V_CTX_CPU_FALLBACK) */
  uint64_t cache_sightings;  /* first sightings recorded instead of claiming a payload (admission, AT2V_CTX_ADMIT_FIRST) */
  uint64_t cache_built;      /* payloads (tables or combs) built */
  uint64_t cache_build_us;   /* device time of the build passes that built something (first build block to the flip) */
  uint64_t cache_record_hits;/* records whose sender came from the cache (launches above small_batch_max verify each
                                record by its own sender's entry, whatever the other records of its chunk) */
  uint64_t experiments;      /* AT2V_EXPERIMENT_* bits compiled into this library (0 in a shipped build) */
  uint64_t host_chunks;      /* chunks staged by the host-buffer calls (at2v_verify_batch / _sharded pipeline) */
} at2v_info;
/* With a sender cache, at2v_get_info first waits for the context's cache work (its build stream, which follows every
 * cached launch and therefore waits for those launches, and whatever each launch's stream ran before them). */
int at2v_get_info(at2v_ctx* ctx, at2v_info* out);

/* ---- multi-GPU, one process per GPU: RCCL all-gather of the verdict bitmap ----
 * A node batch of n records is split by contiguous index range: rank r verifies records
 * [r*per, min(n, (r+1)*per)) with per = ceil(ceil(n/world)/64)*64, i.e. words_per_rank = per/32 verdict words,
 * and one ncclAllGather over xGMI gives every rank the node bitmap, which the apply step (rpc.rs:156-173)
 * consumes. Rank 0 creates the unique id and the caller hands it to the other ranks out of band. */
#define AT2V_UNIQUE_ID_BYTES 128
int at2v_comm_get_unique_id(uint8_t out[AT2V_UNIQUE_ID_BYTES]);
/* Attach an RCCL communicator on ctx's device (single-device contexts only). Collective: blocks until all
 * `world` ranks have called it. The ranks agree on the outcome: if any rank fails its local set-up, every rank
 * returns an error (AT2V_E_PEER on the ranks that did not fail themselves) and no communicator is attached.
 *
 * Failure model of the collective calls below (no rank is ever left waiting inside a collective for a rank that
 * returned early): argument errors are decided from inputs every rank shares (the whole node batch, words_per_rank),
 * so all ranks return before any collective or none does; any later, rank-local failure (allocation, upload, launch)
 * makes that rank join the all-gather anyway with zero verdict words, so its records are verdict 0 on every rank. A
 * device that stops executing work altogether cannot be hidden from its peers. */
int at2v_comm_init_rank(at2v_ctx* ctx, const uint8_t unique_id[AT2V_UNIQUE_ID_BYTES], int rank, int world);
/* Device buffers, asynchronous on hip_stream: verify this rank's n_local records (<= 32*words_per_rank) into
 * d_bitmap + rank*words_per_rank (pad words zeroed), then all-gather (in place) so d_bitmap holds
 * world*words_per_rank words on every rank. Collective: every rank calls it with the same words_per_rank and a
 * valid 4-byte-aligned d_bitmap (AT2V_E_INVALID / AT2V_E_ALIGN otherwise, before the collective). Any other error
 * of this rank (bad record pointers, misalignment, launch failure) is returned AFTER it has joined the all-gather
 * with a zero slice. */
int at2v_verify_shard_gather_device(at2v_ctx* ctx, const uint8_t* d_pk, const uint8_t* d_sig, const uint8_t* d_msg,
                                    size_t msg_bytes, const uint32_t* d_msg_off, size_t n_local,
                                    size_t words_per_rank, uint32_t* d_bitmap, void* hip_stream);
/* Host buffers, synchronous: every rank passes the SAME node batch (at2v_verify_batch layout); each uploads
 * and verifies only its own range, the all-gather fills in the rest, and every rank receives all ceil(n/32)
 * verdict words in record order. Collective. Every rank returns AT2V_OK only if every rank succeeded; otherwise the
 * failing rank returns its error and the others AT2V_E_PEER. */
int at2v_verify_batch_sharded(at2v_ctx* ctx, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg,
                              const uint32_t* msg_off, size_t n, uint32_t* verdicts);


/* ---- ingest/batching queue: the server's verify call site ----
 * Replaces the per-payload verify that sieve/murmur run on num_cpus::get() workers (rpc.rs:125,
 * rpc.rs:275-284 -> rpc.rs:156). Producers submit records; a batch is sealed at max_batch records, when
 * its oldest record is max_delay_us old, or on at2v_queue_flush() — and, with AT2V_QUEUE_EAGER, whenever
 * no batch is in flight (latency mode) — and verified on the GPU asynchronously (depth slots: one
 * filling, up to depth-1 in flight). Verdicts come back in ticket
 * (= submission) order. Thread-safe: any number of producer threads; poll from any thread.
 * A slot's records live in pinned host memory: a batch of up to 1,024 records is read by the kernel from there, a
 * larger one is uploaded first; the kernel writes the verdict words straight into pinned host memory. */
typedef struct at2v_queue at2v_queue;
typedef struct {
  int device;             /* HIP device ordinal */
  at2v_policy policy;
  uint32_t max_batch;     /* records per batch; 0 = 65536 */
  uint32_t max_delay_us;  /* deadline of the oldest pending record; 0 = 1000 */
  uint32_t max_msg_bytes; /* message bytes budgeted per record (slot capacity max_batch x this); 0 = 256 */
  uint32_t depth;         /* batch slots, >= 2; 0 = 3 */
  uint32_t flags;         /* AT2V_QUEUE_EAGER: also seal whenever no batch is in flight; AT2V_QUEUE_SENDER_COMB:
                             per-sender combs (at2v_opts.sender_comb) */
  uint32_t sender_cache;  /* with AT2V_QUEUE_SENDER_COMB: keys the queue's context caches (at2v_opts.sender_cache,
                             1.7 MB of HBM each); 0 = 1024 */
  uint32_t cpu_threads;   /* AT2V_QUEUE_CPU / AT2V_QUEUE_CPU_FALLBACK: host threads (0 = every usable CPU) */
} at2v_queue_opts;
#define AT2V_QUEUE_EAGER 1u
#define AT2V_QUEUE_SENDER_COMB 2u /* the queue's context gets a sender cache (sender_cache keys) with sender_comb = 1 */
#define AT2V_QUEUE_CPU 4u         /* batches verified by the CPU backend (a context with num_gpus = 0): no device */
#define AT2V_QUEUE_CPU_FALLBACK 8u /* a batch whose launch or completion fails on the device is verified on the CPU
                                     backend instead (the slot's records are in host memory); same verdicts */
typedef struct {
  uint64_t submitted, completed, batches, failed_batches;
  double mean_batch;           /* records per completed batch */
  double p50_us, p99_us, max_us; /* submit -> verdict published, per record (since create / reset) */
  uint64_t cpu_fallbacks;        /* AT2V_QUEUE_CPU_FALLBACK: batches the device failed and the CPU backend verified */
} at2v_queue_stats;
int at2v_queue_create(const at2v_queue_opts* opts, at2v_queue** out);
void at2v_queue_destroy(at2v_queue* q); /* seals and completes everything submitted, then frees */
/* n records in the at2v_verify_batch layout; *first_ticket receives the ticket of record 0 (the call's
 * records get consecutive tickets). Blocks only while every slot is busy (backpressure). */
int at2v_queue_submit(at2v_queue* q, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg,
                      const uint32_t* msg_off, size_t n, uint64_t* first_ticket);
int at2v_queue_flush(at2v_queue* q);
/* Up to max completed (ticket, verdict) pairs in ticket order, waiting up to timeout_us for the first.
 * verdict: 1 valid, 0 invalid, 0xff the batch failed on the device. Returns the count (>= 0) or < 0. */
long at2v_queue_poll(at2v_queue* q, uint64_t* tickets, uint8_t* verdicts, size_t max, uint32_t timeout_us);
int at2v_queue_get_stats(at2v_queue* q, at2v_queue_stats* out);
int at2v_queue_reset_latency(at2v_queue* q);

/* ---- record packer: SendAssetRequest fields -> verify records ----
 * Mirrors the server's decode of SendAssetRequest (at2.proto:10-16) at rpc.rs:264-281: recipient, then
 * sender, then signature, each bincode-decoded; M = bincode(ThinTransaction{recipient, amount})
 * (src/lib.rs:14-22, signed at src/client.rs:77-78). `wire` selects how drop's PublicKey/Signature
 * serialise (not in the tree): AT2V_WIRE_BYTES = u64le length prefix + bytes (default assumption),
 * AT2V_WIRE_ARRAY = raw bytes. Curve-point validity is NOT checked here (at2v_decode_points, and V2 of
 * the verify kernel for the sender). */
typedef struct {
  const uint8_t* sender;
  size_t sender_len;
  uint32_t sequence;
  const uint8_t* recipient;
  size_t recipient_len;
  uint64_t amount;
  const uint8_t* signature;
  size_t signature_len;
} at2v_send_asset_request;
enum { AT2V_WIRE_BYTES = 0, AT2V_WIRE_ARRAY = 1 };
enum { AT2V_PACK_OK = 0, AT2V_PACK_BAD_RECIPIENT = 1, AT2V_PACK_BAD_SENDER = 2, AT2V_PACK_BAD_SIGNATURE = 3 };
/* pk_out n x 32, sig_out n x 64, recipient_out n x 32, msg_out n x (48 | 40) bytes, msg_off_out n + 1,
 * status_out n. A record that fails to decode keeps its index (zero key/signature, empty message).
 * Returns the number of records with status AT2V_PACK_OK, or < 0. */
long at2v_pack_send_asset(const at2v_send_asset_request* req, size_t n, int wire, uint8_t* pk_out, uint8_t* sig_out,
                          uint8_t* msg_out, uint32_t* msg_off_out, uint8_t* recipient_out, uint8_t* status_out);

/* Curve-point decoding on the GPU: bit i of valid_words = 1 iff pts[i] (32 bytes) decodes under
 * curve25519-dalek CompressedEdwardsY::decompress — what bincode-deserialising a
 * drop PublicKey checks at rpc.rs:265/269. Host buffers, synchronous, ctx's first device. */
int at2v_decode_points(at2v_ctx* ctx, const uint8_t* pts, size_t n, uint32_t* valid_words);

/* ---- ledger apply: what the server does with verified payloads ----
 * Accounts (accounts/mod.rs, account.rs), the 10-entry recent-transactions log (recent_transactions.rs)
 * and the deliver/apply loop of Service::spawn (rpc.rs:149-211), with the reference's quirks: an
 * Underflow still consumes the sequence, every account error is retried, payloads are processed in
 * descending (sequence, sender, recipient, amount) order per pass, TTL expiry (60 s) marks Failure but
 * does not skip processing. Not thread-safe. */
typedef struct at2v_ledger at2v_ledger;
enum { AT2V_TX_OK = 0, AT2V_TX_INCONSECUTIVE_SEQUENCE = 1, AT2V_TX_OVERFLOW = 2, AT2V_TX_UNDERFLOW = 3 };
enum { AT2V_TX_PENDING = 0, AT2V_TX_SUCCESS = 1, AT2V_TX_FAILURE = 2 };
typedef struct {
  uint64_t timestamp_us;
  uint8_t sender[32];
  uint32_t sender_sequence;
  uint8_t recipient[32];
  uint64_t amount;
  int32_t state; /* AT2V_TX_PENDING / SUCCESS / FAILURE */
} at2v_full_transaction;
typedef struct {
  uint64_t delivered; /* records whose verdict bit was 1 */
  uint64_t rejected;  /* records whose verdict bit was 0 (never delivered) */
  uint64_t applied;   /* transfers that succeeded during this call */
  uint64_t requeued;  /* payloads still pending after the call (account errors are retried later) */
  uint64_t expired;   /* TTL-expired payloads marked Failure during this call */
  uint64_t passes;    /* passes of the apply loop */
} at2v_apply_stats;
int at2v_ledger_create(at2v_ledger** out);
void at2v_ledger_destroy(at2v_ledger* l);
int at2v_ledger_balance(const at2v_ledger* l, const uint8_t pk[32], uint64_t* out);
int at2v_ledger_last_sequence(const at2v_ledger* l, const uint8_t pk[32], uint32_t* out);
/* AccountsHandler::transfer: returns AT2V_TX_OK or an AT2V_TX_* error (>0), < 0 on bad arguments. */
int at2v_ledger_transfer(at2v_ledger* l, const uint8_t sender[32], uint32_t sequence, const uint8_t recipient[32],
                         uint64_t amount);
int at2v_ledger_recent_put(at2v_ledger* l, const uint8_t sender[32], uint32_t sequence, const uint8_t recipient[32],
                           uint64_t amount, uint64_t now_us);
long at2v_ledger_recent_get(const at2v_ledger* l, at2v_full_transaction* out, size_t max);
/* One delivered batch: records i with verdict bit i set (verdicts NULL = all) enter the apply loop. */
int at2v_ledger_deliver(at2v_ledger* l, const uint8_t* sender, const uint32_t* sequence, const uint8_t* recipient,
                        const uint64_t* amount, const uint32_t* verdicts, size_t n, uint64_t now_us,
                        at2v_apply_stats* stats);
long at2v_ledger_pending(const at2v_ledger* l);

#ifdef __cplusplus
}
#endif
#endif /* AT2V_H */
