/*
 * crosscheck.c — pins the oracle (TEST INFRASTRUCTURE, runs only in the build container).
 *
 * 1. RFC 8032 §7.1 TEST 1-3 known answers (public key + signature from the secret seed).
 * 2. Oracle signer == OpenSSL 3.0.2 signer (Ed25519 is deterministic).
 * 3. Verdicts: oracle DALEK_V1 policy == OpenSSL 3.0.2 EVP_DigestVerify, and oracle
 *    LIBSODIUM_1_0_18 policy == libsodium 1.0.18 crypto_sign_verify_detached, on every
 *    record of every fixture set (valid, adversarial, edge, ragged lengths, AT2 config 1).
 * 4. Writes the fixture sets to <outdir>/<name>.bin (format: tests/golden/README.md).
 *
 * Neither OpenSSL nor libsodium travels to the GPU box: only the .bin fixtures do.
 * Build + run: make -C oracle fixtures
 */
#include <dlfcn.h>
#include <openssl/evp.h>
#include <openssl/opensslv.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ed25519_oracle.h"

static int (*sodium_init_p)(void);
static int (*sodium_verify_p)(const unsigned char*, const unsigned char*, unsigned long long, const unsigned char*);

static int openssl_verify(const uint8_t* pk, const uint8_t* sig, const uint8_t* m, size_t len) {
  EVP_PKEY* key = EVP_PKEY_new_raw_public_key(EVP_PKEY_ED25519, NULL, pk, 32);
  if (!key) return 0;
  EVP_MD_CTX* ctx = EVP_MD_CTX_new();
  int ok = 0;
  if (EVP_DigestVerifyInit(ctx, NULL, NULL, NULL, key) == 1) ok = EVP_DigestVerify(ctx, sig, 64, m, len) == 1;
  EVP_MD_CTX_free(ctx);
  EVP_PKEY_free(key);
  return ok;
}

static int openssl_sign(const uint8_t seed[32], const uint8_t* m, size_t len, uint8_t sig[64], uint8_t pk[32]) {
  EVP_PKEY* key = EVP_PKEY_new_raw_private_key(EVP_PKEY_ED25519, NULL, seed, 32);
  if (!key) return 0;
  size_t pl = 32, sl = 64;
  EVP_PKEY_get_raw_public_key(key, pk, &pl);
  EVP_MD_CTX* ctx = EVP_MD_CTX_new();
  int ok = EVP_DigestSignInit(ctx, NULL, NULL, NULL, key) == 1 && EVP_DigestSign(ctx, sig, &sl, m, len) == 1;
  EVP_MD_CTX_free(ctx);
  EVP_PKEY_free(key);
  return ok;
}

static int sodium_verify(const uint8_t* pk, const uint8_t* sig, const uint8_t* m, size_t len) {
  return sodium_verify_p(sig, m, len, pk) == 0;
}

static void hex2bin(const char* h, uint8_t* out, size_t n) {
  for (size_t i = 0; i < n; ++i) {
    unsigned v;
    sscanf(h + 2 * i, "%2x", &v);
    out[i] = (uint8_t)v;
  }
}

typedef struct {
  size_t n, cap_msg, used_msg;
  uint8_t *pk, *sig, *msg, *dalek, *sodium, *cls;
  uint32_t* off;
} fixset;

static void fs_init(fixset* f, size_t n, size_t cap_msg) {
  memset(f, 0, sizeof *f);
  f->pk = calloc(n, 32);
  f->sig = calloc(n, 64);
  f->msg = calloc(cap_msg ? cap_msg : 1, 1);
  f->off = calloc(n + 1, 4);
  f->dalek = calloc(n, 1);
  f->sodium = calloc(n, 1);
  f->cls = calloc(n, 1);
  f->cap_msg = cap_msg;
}

static void fs_push(fixset* f, const uint8_t* pk, const uint8_t* sig, const uint8_t* m, size_t len, uint8_t cls) {
  if (f->used_msg + len > f->cap_msg) {
    fprintf(stderr, "fixture msg capacity\n");
    exit(2);
  }
  memcpy(f->pk + 32 * f->n, pk, 32);
  memcpy(f->sig + 64 * f->n, sig, 64);
  memcpy(f->msg + f->used_msg, m, len);
  f->off[f->n] = (uint32_t)f->used_msg;
  f->used_msg += len;
  f->cls[f->n] = cls;
  f->n++;
  f->off[f->n] = (uint32_t)f->used_msg;
}

static long g_mismatch = 0;

/* computes verdicts with all engines, asserts agreement, writes file */
static void fs_finish(fixset* f, const char* dir, const char* name) {
  long acc_d = 0, acc_s = 0;
  for (size_t i = 0; i < f->n; ++i) {
    const uint8_t* m = f->msg + f->off[i];
    size_t len = f->off[i + 1] - f->off[i];
    int od = oracle_verify(f->pk + 32 * i, f->sig + 64 * i, m, len, ORACLE_POLICY_DALEK_V1);
    int os = oracle_verify(f->pk + 32 * i, f->sig + 64 * i, m, len, ORACLE_POLICY_LIBSODIUM_1_0_18);
    int ssl = openssl_verify(f->pk + 32 * i, f->sig + 64 * i, m, len);
    int na = sodium_verify(f->pk + 32 * i, f->sig + 64 * i, m, len);
    if (od != ssl || os != na) {
      if (g_mismatch < 20)
        fprintf(stderr, "MISMATCH %s[%zu] cls=%d oracle_dalek=%d openssl=%d oracle_sodium=%d libsodium=%d\n", name, i,
                f->cls[i], od, ssl, os, na);
      ++g_mismatch;
    }
    f->dalek[i] = (uint8_t)ssl;
    f->sodium[i] = (uint8_t)na;
    acc_d += ssl;
    acc_s += na;
  }
  char path[1024];
  snprintf(path, sizeof path, "%s/%s.bin", dir, name);
  FILE* fp = fopen(path, "wb");
  if (!fp) {
    perror(path);
    exit(2);
  }
  uint32_t hdr[4] = {0x56325441u /* "AT2V" */, 1u, (uint32_t)f->n, (uint32_t)f->used_msg};
  fwrite(hdr, 4, 4, fp);
  fwrite(f->pk, 32, f->n, fp);
  fwrite(f->sig, 64, f->n, fp);
  fwrite(f->off, 4, f->n + 1, fp);
  fwrite(f->msg, 1, f->used_msg, fp);
  fwrite(f->dalek, 1, f->n, fp);
  fwrite(f->sodium, 1, f->n, fp);
  fwrite(f->cls, 1, f->n, fp);
  fclose(fp);
  printf("%-14s n=%6zu msg_bytes=%8zu accept(dalek/openssl)=%6ld accept(libsodium)=%6ld\n", name, f->n, f->used_msg,
         acc_d, acc_s);
}

int main(int argc, char** argv) {
  const char* dir = argc > 1 ? argv[1] : "tests/golden";
  void* so = dlopen("/opt/conda/lib/libsodium.so", RTLD_NOW);
  if (!so) {
    fprintf(stderr, "libsodium not found: %s\n", dlerror());
    return 2;
  }
  sodium_init_p = (int (*)(void))dlsym(so, "sodium_init");
  sodium_verify_p = (int (*)(const unsigned char*, const unsigned char*, unsigned long long,
                             const unsigned char*))dlsym(so, "crypto_sign_verify_detached");
  const char* (*sodium_ver)(void) = (const char* (*)(void))dlsym(so, "sodium_version_string");
  if (!sodium_init_p || !sodium_verify_p || sodium_init_p() < 0) return 2;
  printf("openssl: %s | libsodium: %s\n", OPENSSL_VERSION_TEXT, sodium_ver ? sodium_ver() : "?");

  /* 1. RFC 8032 §7.1 TEST 1-3 */
  static const char* rfc[3][4] = {
      {"9d61b19deffd5a60ba844af492ec2cc44449c5697b326919703bac031cae7f60",
       "d75a980182b10ab7d54bfed3c964073a0ee172f3daa62325af021a68f707511a", "",
       "e5564300c360ac729086e2cc806e828a84877f1eb8e5d974d873e065224901555fb8821590a33bacc61e39701cf9b46bd25bf5f0595bbe2"
       "4655141438e7a100b"},
      {"4ccd089b28ff96da9db6c346ec114e0f5b8a319f35aba624da8cf6ed4fb8a6fb",
       "3d4017c3e843895a92b70aa74d1b7ebc9c982ccf2ec4968cc0cd55f12af4660c", "72",
       "92a009a9f0d4cab8720e820b5f642540a2b27b5416503f8fb3762223ebdb69da085ac1e43e15996e458f3613d0f11d8c387b2eaeb4302aee"
       "b00d291612bb0c00"},
      {"c5aa8df43f9f837bedb7442f31dcb7b166d38535076f094b85ce3a2e0b4458f7",
       "fc51cd8e6218a1a38da47ed00230f0580816ed13ba3303ac5deb911548908025", "af82",
       "6291d657deec24024827e69c3abe01a30ce548a284743a445e3680d7db5ac3ac18ff9b538d16f290ae67f760984dc6594a7c15e9716ed28d"
       "c027beceea1ec40a"}};
  fixset rfcset;
  fs_init(&rfcset, 3, 16);
  int fails = 0;
  for (int t = 0; t < 3; ++t) {
    uint8_t seed[32], pk[32], sig[64], m[2], opk[32], osig[64], spk[32], ssig[64];
    size_t mlen = strlen(rfc[t][2]) / 2;
    hex2bin(rfc[t][0], seed, 32);
    hex2bin(rfc[t][1], pk, 32);
    hex2bin(rfc[t][2], m, mlen);
    hex2bin(rfc[t][3], sig, 64);
    oracle_public_key(seed, opk);
    oracle_sign(seed, m, mlen, osig);
    openssl_sign(seed, m, mlen, ssig, spk);
    int ok = !memcmp(pk, opk, 32) && !memcmp(sig, osig, 64) && !memcmp(pk, spk, 32) && !memcmp(sig, ssig, 64) &&
             oracle_verify(pk, sig, m, mlen, 0) && openssl_verify(pk, sig, m, mlen);
    printf("RFC8032 TEST %d: %s\n", t + 1, ok ? "ok" : "FAIL");
    fails += !ok;
    fs_push(&rfcset, pk, sig, m, mlen, 0);
  }
  fs_finish(&rfcset, dir, "rfc8032");

  /* 2. signer agreement on generated records */
  {
    const size_t n = 256;
    uint8_t *pk = malloc(32 * n), *sig = malloc(64 * n), *msg = malloc(100 * n);
    oracle_gen_records(0x4154325fULL, 0, n, 100, pk, sig, msg, 8);
    int bad = 0;
    for (size_t i = 0; i < n; ++i) {
      uint8_t seed[32], spk[32], ssig[64];
      oracle_gen_seed(0x4154325fULL, i, seed);
      openssl_sign(seed, msg + 100 * i, 100, ssig, spk);
      bad += memcmp(spk, pk + 32 * i, 32) != 0 || memcmp(ssig, sig + 64 * i, 64) != 0;
    }
    printf("signer agreement oracle vs openssl: %zu/%zu\n", n - (size_t)bad, n);
    fails += bad != 0;
    free(pk);
    free(sig);
    free(msg);
  }

  /* 3a. config 1: AT2 transactions */
  {
    fixset f;
    fs_init(&f, 4096, 4096 * 48);
    uint8_t *pk = malloc(32 * 4096), *sig = malloc(64 * 4096), *msg = malloc(48 * 4096);
    uint32_t *snd = malloc(4 * 4096), *seq = malloc(4 * 4096);
    oracle_gen_at2_transactions(0x4154325fULL, pk, sig, msg, snd, seq);
    for (size_t i = 0; i < 4096; ++i) fs_push(&f, pk + 32 * i, sig + 64 * i, msg + 48 * i, 48, 0);
    fs_finish(&f, dir, "at2_cfg1");
    free(pk); free(sig); free(msg); free(snd); free(seq);
  }

  /* 3b. adversarial (config 4 mix), 100-byte messages */
  {
    const size_t n = 8192;
    fixset f;
    fs_init(&f, n, n * 100);
    uint8_t *pk = malloc(32 * n), *sig = malloc(64 * n), *msg = malloc(100 * n), *cls = malloc(n);
    oracle_gen_adversarial(0x4154325fULL, 0, n, 100, pk, sig, msg, cls, 8);
    for (size_t i = 0; i < n; ++i) fs_push(&f, pk + 32 * i, sig + 64 * i, msg + 100 * i, 100, cls[i]);
    fs_finish(&f, dir, "adversarial");
    free(pk); free(sig); free(msg); free(cls);
  }

  /* 3c. edge cases: every small-order encoding as A and as R, s = 0 / l-1 / l / 2^253 ... */
  {
    fixset f;
    fs_init(&f, 4096, 4096 * 64);
    uint8_t m[64];
    oracle_gen_msg(7, 7, m, 64);
    uint8_t lb[32] = {0xed, 0xd3, 0xf5, 0x5c, 0x1a, 0x63, 0x12, 0x58, 0xd6, 0x9c, 0xf7, 0xa2, 0xde, 0xf9, 0xde, 0x14,
                      0,    0,    0,    0,    0,    0,    0,    0,    0,    0,    0,    0,    0,    0,    0,    0x10};
    for (int a = 0; a < 14; ++a) {
      uint8_t A[32];
      oracle_small_order_encoding(a, A);
      /* A small order, S in {0, 1, 2, 8, random}, R = [S]B: accept iff [k]A == 0 */
      for (int sv = 0; sv < 24; ++sv) {
        uint8_t S[32] = {0}, sig[64];
        if (sv < 4) S[0] = (uint8_t)(sv == 3 ? 8 : sv);
        else {
          uint8_t h[64];
          oracle_sha512(&m[sv], 8, h);
          memcpy(S, h, 32);
          S[31] &= 0x0f;
        }
        oracle_scalarmult_base(S, sig);
        memcpy(sig + 32, S, 32);
        fs_push(&f, A, sig, m, (size_t)sv, 6);
      }
      /* R small order too: R = each of the 14 encodings, S = 0 */
      for (int r = 0; r < 14; ++r) {
        uint8_t sig[64] = {0};
        oracle_small_order_encoding(r, sig);
        fs_push(&f, A, sig, m, 32, 5);
      }
    }
    /* scalar boundary: valid sig with S replaced by l-1, l, l+1, 2^252, 2^253-1, 2^255, all-ones */
    {
      uint8_t seed[32], pk[32], sig[64];
      oracle_gen_seed(99, 1, seed);
      oracle_public_key(seed, pk);
      oracle_sign(seed, m, 64, sig);
      fs_push(&f, pk, sig, m, 64, 0);
      for (int v = 0; v < 8; ++v) {
        uint8_t s2[64];
        memcpy(s2, sig, 64);
        uint8_t* S = s2 + 32;
        switch (v) {
          case 0: memcpy(S, lb, 32); S[0] -= 1; break;
          case 1: memcpy(S, lb, 32); break;
          case 2: memcpy(S, lb, 32); S[0] += 1; break;
          case 3: memset(S, 0, 32); S[31] = 0x10; break;
          case 4: memset(S, 0xff, 32); S[31] = 0x1f; break;
          case 5: memset(S, 0, 32); S[31] = 0x80; break;
          case 6: memset(S, 0xff, 32); break;
          case 7: memset(S, 0, 32); break;
        }
        fs_push(&f, pk, s2, m, 64, 3);
      }
    }
    /* non-canonical R for a point that the equation does hit: A = identity, S = s, R' = [s]B; R given as
     * y+p when y([s]B) < 19 is unreachable, so use the identity/-1 points whose y has a y+p alias */
    {
      uint8_t one[32] = {1};
      for (int v = 0; v < 4; ++v) {
        uint8_t sig[64] = {0};
        if (v == 0) sig[0] = 1;                                                      /* canonical identity */
        if (v == 1) { sig[0] = 1; sig[31] = 0x80; }                                  /* -0 */
        if (v == 2) { memset(sig, 0xff, 32); sig[0] = 0xee; sig[31] = 0x7f; }        /* p+1 */
        if (v == 3) { memset(sig, 0xff, 32); sig[0] = 0xee; sig[31] = 0xff; }        /* p+1, sign */
        fs_push(&f, one, sig, m, 0, 5);
      }
    }
    /* A non-canonical aliases of real keys are unreachable (y < 19 only for torsion); A off-curve sweep */
    for (int y = 0; y < 64; ++y) {
      uint8_t A[32] = {0}, seed[32], sig[64];
      A[0] = (uint8_t)y;
      A[31] = (uint8_t)((y & 1) << 7);
      oracle_gen_seed(5, (uint64_t)y, seed);
      oracle_sign(seed, m, 16, sig);
      fs_push(&f, A, sig, m, 16, 7);
    }
    fs_finish(&f, dir, "edge");
  }

  /* 3d. ragged message lengths 0..319 (crosses the 1/2/3 SHA-512 block boundaries at 47/48, 175/176, 303/304) */
  {
    const size_t n = 320;
    fixset f;
    fs_init(&f, n, n * 320);
    uint8_t* m = malloc(320);
    for (size_t i = 0; i < n; ++i) {
      uint8_t seed[32], pk[32], sig[64];
      oracle_gen_seed(11, i, seed);
      oracle_gen_msg(11, i, m, i);
      oracle_public_key(seed, pk);
      oracle_sign(seed, m, i, sig);
      if (i % 5 == 4) sig[i % 64] ^= 0x10; /* every 5th one corrupted */
      fs_push(&f, pk, sig, m, i, i % 5 == 4 ? 1 : 0);
    }
    fs_finish(&f, dir, "ragged");
    free(m);
  }

  printf("verdict mismatches: %ld; other failures: %d\n", g_mismatch, fails);
  return (g_mismatch || fails) ? 1 : 0;
}
