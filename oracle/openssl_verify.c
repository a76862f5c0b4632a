/*
 * openssl_verify.c — CPU BASELINE leg (test/bench infrastructure; never the shipped path).
 *
 * "CPU baseline: OpenSSL libcrypto Ed25519 verify if present on the GPU box, else the build's C++
 * oracle". This wraps OpenSSL 3.x EVP_DigestVerify (EVP_PKEY_ED25519, one-shot) over a batch with one pthread per
 * core, static index partition, so bench.py can time a production-grade CPU Ed25519 beside the oracle. OpenSSL 3.0.2
 * matches the dalek-1.x verdicts on every edge class SURVEY Appendix B probed; it is a stand-in for the reference's
 * rayon ed25519-dalek path, which cannot be built here.
 */
#include <openssl/evp.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>

static int verify_one(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, size_t len) {
  EVP_PKEY* key = EVP_PKEY_new_raw_public_key(EVP_PKEY_ED25519, NULL, pk, 32);
  if (!key) return 0;
  EVP_MD_CTX* ctx = EVP_MD_CTX_new();
  int ok = 0;
  if (ctx && EVP_DigestVerifyInit(ctx, NULL, NULL, NULL, key) == 1)
    ok = EVP_DigestVerify(ctx, sig, 64, msg, len) == 1;
  EVP_MD_CTX_free(ctx);
  EVP_PKEY_free(key);
  return ok;
}

typedef struct {
  const uint8_t *pk, *sig, *msg;
  const uint32_t* off;
  uint8_t* out;
  size_t lo, hi;
} job_t;

static void* worker(void* p) {
  job_t* j = (job_t*)p;
  for (size_t i = j->lo; i < j->hi; ++i)
    j->out[i] = (uint8_t)verify_one(j->pk + 32 * i, j->sig + 64 * i, j->msg + j->off[i], j->off[i + 1] - j->off[i]);
  return NULL;
}

/* out[i] = 1 iff record i verifies; returns 0, or -1 if a thread could not be started */
int ossl_verify_batch(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, const uint32_t* off, size_t n,
                      int threads, uint8_t* out) {
  if (threads < 1) threads = 1;
  if ((size_t)threads > n) threads = n ? (int)n : 1;
  pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
  job_t* jobs = (job_t*)calloc((size_t)threads, sizeof(job_t));
  if (!th || !jobs) {
    free(th);
    free(jobs);
    return -1;
  }
  int rc = 0, started = 0;
  for (int t = 0; t < threads; ++t) {
    jobs[t] = (job_t){pk, sig, msg, off, out, n * (size_t)t / (size_t)threads, n * (size_t)(t + 1) / (size_t)threads};
    if (pthread_create(&th[t], NULL, worker, &jobs[t]) != 0) {
      rc = -1;
      break;
    }
    ++started;
  }
  for (int t = 0; t < started; ++t) pthread_join(th[t], NULL);
  free(th);
  free(jobs);
  return rc;
}
