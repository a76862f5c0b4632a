/*
 * ed25519_oracle.h — CPU ORACLE for the at2v hot path (TEST INFRASTRUCTURE ONLY).
 *
 * This is a plain-C restatement of the verify semantics at2-node relies on:
 * drop::crypto::sign (git dep, Cargo.toml:9, no rev pinned) → ed25519-dalek 1.x
 * `PublicKey::verify` over curve25519-dalek 3.x + sha2 0.9 (SURVEY.md §0.3,
 * Appendix A steps V1–V6). The arithmetic lives in that third-party dependency,
 * which is NOT in /root/reference; the restatement follows its published
 * algorithm (NAF-5 variable-base / NAF-8 fixed-base vartime double-scalar mult).
 *
 * Reference call sites this oracle stands behind:
 *   - signing:   src/client.rs:77-78   (KeyPair::sign over bincode(ThinTransaction))
 *   - decode A:  src/bin/server/rpc.rs:269  (PublicKey deserialize = decompress)
 *   - decode sig: src/bin/server/rpc.rs:281
 *   - verify:    inside sieve/murmur on every payload broadcast at rpc.rs:275-284,
 *                consumed (already verified) at rpc.rs:156-173.
 *
 * Parity pinning: the reference's own tests hold no known-answer vectors for this
 * boundary. The oracle is pinned instead against OpenSSL
 * 3.0.2 libcrypto (same verdicts as dalek-1.x `verify` on every probed edge class,
 * SURVEY Appendix B) and RFC 8032 §7.1 vectors; libsodium 1.0.18 pins the strict
 * policy. See oracle/crosscheck.c and tests/golden/.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this code. It is never part of the shipped verify path.
 */
#ifndef AT2V_ED25519_ORACLE_H
#define AT2V_ED25519_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* policies: identical numbering to include/at2v.h */
#define ORACLE_POLICY_DALEK_V1 0
#define ORACLE_POLICY_LIBSODIUM_1_0_18 1

void oracle_sha512(const uint8_t* in, size_t len, uint8_t out[64]);

/* 1 = accept, 0 = reject. */
int oracle_verify(const uint8_t pk[32], const uint8_t sig[64], const uint8_t* msg, size_t len, int policy);

/* verdicts: ceil(n/32) words, bit i%32 of word i/32 set iff record i valid.
 * msg_off has n+1 entries. threads <= 0 → 1. */
void oracle_verify_batch(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, const uint32_t* msg_off,
                         size_t n, int policy, uint32_t* verdicts, int threads);

/* RFC 8032 key generation / signing from a 32-byte seed. */
void oracle_public_key(const uint8_t seed[32], uint8_t pk[32]);
void oracle_sign(const uint8_t seed[32], const uint8_t* msg, size_t len, uint8_t sig[64]);

/* out = enc([s]B) for an arbitrary 256-bit little-endian scalar s (not reduced). */
void oracle_scalarmult_base(const uint8_t s[32], uint8_t out[32]);
/* out = enc(dec(p) + dec(q)) with dalek decode rules; returns 0 if either fails to decode. */
int oracle_point_add(const uint8_t p[32], const uint8_t q[32], uint8_t out[32]);
/* out = enc([s]dec(p)); returns 0 if p fails to decode. */
int oracle_scalarmult(const uint8_t s[32], const uint8_t p[32], uint8_t out[32]);
/* 1 if the 32-byte encoding decodes under dalek rules. */
int oracle_decompress_ok(const uint8_t p[32]);

/* scalar helpers (mod l = 2^252 + 27742317777372353535851937790883648493) */
void oracle_sc_reduce64(const uint8_t in[64], uint8_t out[32]);
int oracle_sc_is_canonical(const uint8_t s[32]);
/* out = (a*b + c) mod l */
void oracle_sc_muladd(const uint8_t a[32], const uint8_t b[32], const uint8_t c[32], uint8_t out[32]);

/* Deterministic synthetic record generator.
 * seed_i = SHA-512("at2v/seed" || u64le(cfg_seed) || u64le(i))[0:32]
 * msg kind 0 ("cfg2"): M_i = SHA-512 counter stream of ("at2v/msg" || u64le(cfg_seed) || u64le(i) || u64le(ctr)),
 *                       truncated to msg_len bytes.
 * Writes pk[n*32], sig[n*64], msg[n*msg_len] for records first..first+n-1 (msg_off is implicit: i*msg_len). */
void oracle_gen_seed(uint64_t cfg_seed, uint64_t i, uint8_t seed[32]);
void oracle_gen_msg(uint64_t cfg_seed, uint64_t i, uint8_t* msg, size_t msg_len);
void oracle_gen_records(uint64_t cfg_seed, uint64_t first, size_t n, size_t msg_len, uint8_t* pk, uint8_t* sig,
                        uint8_t* msg, int threads);

/* AT2 ThinTransaction message: bincode(ThinTransaction{recipient, amount}) (src/lib.rs:14-22)
 * = u64le(32) || recipient[32] || u64le(amount)  (48 bytes; SURVEY §8(a) a1 layout). */
size_t oracle_thin_transaction(const uint8_t recipient[32], uint64_t amount, uint8_t out[48]);

/* Config 1: 4096 AT2 send-asset transactions (64 senders x sequences 1..64), 48-byte messages. */
void oracle_gen_at2_transactions(uint64_t cfg_seed, uint8_t* pk, uint8_t* sig, uint8_t* msg, uint32_t* sender,
                                 uint32_t* sequence);
/* Config 4: adversarial mix; cls[i] = class id 0..7 (0 = untouched valid signature). */
void oracle_gen_adversarial(uint64_t cfg_seed, uint64_t first, size_t n, size_t msg_len, uint8_t* pk, uint8_t* sig,
                            uint8_t* msg, uint8_t* cls, int threads);
/* idx 0..13: the 14 encodings of the 8 small-order points (7 y values x sign bit). */
void oracle_small_order_encoding(int idx, uint8_t out[32]);

#ifdef __cplusplus
}
#endif
#endif
