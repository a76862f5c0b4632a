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

typedef struct at2v_ctx at2v_ctx; /* opaque: device(s), streams, scratch, staging buffers, RCCL comms */

typedef enum {
  AT2V_POLICY_DALEK_V1 = 0,         /* ed25519-dalek 1.x PublicKey::verify (the reference; default) */
  AT2V_POLICY_LIBSODIUM_1_0_18 = 1  /* + libsodium 1.0.18 pre-rejects: A non-canonical / small order, R small order */
} at2v_policy;

typedef struct {
  int device;         /* first HIP device ordinal (default 0) */
  int num_gpus;       /* devices device..device+num_gpus-1 share each host batch by index range; 0 or 1 = one GPU */
  at2v_policy policy; /* verdict semantics */
} at2v_opts;

enum {
  AT2V_OK = 0,
  AT2V_E_INVALID = -1,  /* bad argument (NULL pointer, n too large, ...) */
  AT2V_E_NODEVICE = -2, /* no usable gfx950 device / library built without the HIP kernels */
  AT2V_E_HIP = -3,      /* HIP runtime error */
  AT2V_E_OOM = -4,      /* device or host allocation failed */
  AT2V_E_ALIGN = -5,    /* device pointer not 16-byte aligned (pk, sig) or 4-byte aligned (offsets, verdicts) */
  AT2V_E_RCCL = -6      /* RCCL communicator / collective failure (multi-GPU contexts) */
};

/* Create / destroy a context. opts may be NULL (device 0, one GPU, DALEK_V1). Replaces nothing in the
 * reference directly: it owns what drop's SystemManager::run(.., num_cpus::get()) workers did
 * implicitly (rpc.rs:124-125). A context is not thread-safe: one thread at a time. */
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

/* Batch verify on device-resident buffers of ctx's first device, asynchronously on `hip_stream`
 * (a hipStream_t; NULL = the null stream). Same layout as at2v_verify_batch; msg_bytes = size of the
 * msg buffer in bytes (>= msg_off[n]); d_pk/d_sig 16-byte aligned, d_msg_off/d_verdicts 4-byte aligned.
 * Returns after the launch; results are valid once the stream reaches this point. */
int at2v_verify_batch_device(at2v_ctx* ctx, const uint8_t* d_pk, const uint8_t* d_sig, const uint8_t* d_msg,
                             size_t msg_bytes, const uint32_t* d_msg_off, size_t n, uint32_t* d_verdicts,
                             void* hip_stream);

/* One signature, synchronous: 1 = valid, 0 = invalid, < 0 = error. The drop-in for the
 * per-signature `verify(&message, &public_key)` shape; runs a 1-record batch on a
 * process-wide default context (device 0, DALEK_V1), serialised by an internal mutex. */
int at2v_verify_one(const uint8_t pk[32], const uint8_t sig[64], const uint8_t* msg, size_t len);

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

/* RFC 8032 signing of host messages under 32-byte seeds (host buffers, synchronous). pk_out n x 32,
 * sig_out n x 64. The GPU counterpart of KeyPair::sign (drop), used by tests and the bench generator. */
int at2v_sign_batch(at2v_ctx* ctx, const uint8_t* seeds, const uint8_t* msg, const uint32_t* msg_off, size_t n,
                    uint8_t* pk_out, uint8_t* sig_out);

/* Introspection for benches: kernel geometry actually used by the last verify launch. */
typedef struct {
  int num_gpus;
  int grid_blocks;     /* per device */
  int block_threads;
  int waves_per_cu;    /* resident waves per CU admitted by the kernel's register/LDS use */
  int cus;             /* compute units of the first device */
  int vgprs;           /* VGPRs per lane of the verify kernel (from the code object) */
} at2v_info;
int at2v_get_info(at2v_ctx* ctx, at2v_info* out);

#ifdef __cplusplus
}
#endif
#endif /* AT2V_H */
