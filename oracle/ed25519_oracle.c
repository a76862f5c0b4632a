/*
 * ed25519_oracle.c — CPU ORACLE (test infrastructure; never the shipped path).
 *
 * Restates, in plain C99 + unsigned __int128, the verify algorithm at2-node gets
 * from drop::crypto::sign → ed25519-dalek 1.x `PublicKey::verify`
 * (SURVEY.md §0.3 and Appendix A, steps V1–V6). Nothing here is copied from any
 * implementation; it is written from the published algorithm:
 *   V1 s = LE256(S), reject if s >= l                      (Signature parse, check_scalar)
 *   V2 A decode: y = LE255(A) mod p (y >= p NOT rejected), (ok,x) = sqrt_ratio_i(y^2-1, d y^2+1),
 *      reject if !ok, x := -x if A[31]>>7 (also for x = 0)  (CompressedEdwardsY::decompress)
 *   V3 k = LE512(SHA-512(R || A || M)) mod l, raw bytes of R and A hashed
 *   V4 R' = [k](-A) + [s]B, cofactorless, vartime NAF-5 (A) / NAF-8 (B) double-base
 *   V5 enc(R') canonical; V6 accept iff enc(R') == R bytes.
 * Policy LIBSODIUM_1_0_18 adds libsodium 1.0.18's pre-rejects (Appendix A.4).
 *
 * Field: GF(2^255-19) as 5 x 51-bit limbs (u64), products in unsigned __int128.
 *
 * Parity status: UNPINNED against the reference itself. at2-node holds no vectors for this path and its verify
 * lives in the unvendored, unbuildable drop -> ed25519-dalek dependency. What pins this restatement
 * instead: RFC 8032 §7.1 TEST 1-3, OpenSSL 3.0.2 EVP_DigestVerify (dalek-1.x semantics on every probed edge class)
 * and libsodium 1.0.18 (strict policy), 0 mismatches over 13,220 fixture records (oracle/crosscheck.c,
 * tests/golden/crosscheck.log).
 */
#include "ed25519_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;

/* ------------------------------------------------------------------ SHA-512 */
/* FIPS 180-4 §6.4 */
static const uint64_t SHA512_K[80] = {
    0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL, 0x3956c25bf348b538ULL,
    0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL, 0xd807aa98a3030242ULL, 0x12835b0145706fbeULL,
    0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL, 0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL,
    0xc19bf174cf692694ULL, 0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
    0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL, 0x983e5152ee66dfabULL,
    0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL, 0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL,
    0x06ca6351e003826fULL, 0x142929670a0e6e70ULL, 0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL,
    0x53380d139d95b3dfULL, 0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
    0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL, 0xd192e819d6ef5218ULL,
    0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL, 0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL,
    0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL, 0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL,
    0x682e6ff3d6b2b8a3ULL, 0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
    0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL, 0xca273eceea26619cULL,
    0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL, 0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL,
    0x113f9804bef90daeULL, 0x1b710b35131c471bULL, 0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL,
    0x431d67c49c100d4cULL, 0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL};

typedef struct {
  uint64_t h[8];
  uint8_t buf[128];
  size_t fill;
  uint64_t total;
} sha512_ctx;

static uint64_t ror64(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

static void sha512_block(uint64_t h[8], const uint8_t* p) {
  uint64_t w[80];
  for (int t = 0; t < 16; ++t) {
    uint64_t v = 0;
    for (int b = 0; b < 8; ++b) v = (v << 8) | p[8 * t + b];
    w[t] = v;
  }
  for (int t = 16; t < 80; ++t) {
    uint64_t s0 = ror64(w[t - 15], 1) ^ ror64(w[t - 15], 8) ^ (w[t - 15] >> 7);
    uint64_t s1 = ror64(w[t - 2], 19) ^ ror64(w[t - 2], 61) ^ (w[t - 2] >> 6);
    w[t] = w[t - 16] + s0 + w[t - 7] + s1;
  }
  uint64_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int t = 0; t < 80; ++t) {
    uint64_t S1 = ror64(e, 14) ^ ror64(e, 18) ^ ror64(e, 41);
    uint64_t ch = (e & f) ^ (~e & g);
    uint64_t t1 = hh + S1 + ch + SHA512_K[t] + w[t];
    uint64_t S0 = ror64(a, 28) ^ ror64(a, 34) ^ ror64(a, 39);
    uint64_t mj = (a & b) ^ (a & c) ^ (b & c);
    uint64_t t2 = S0 + mj;
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

static void sha512_init(sha512_ctx* c) {
  static const uint64_t iv[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                                 0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                                 0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
  memcpy(c->h, iv, sizeof iv);
  c->fill = 0;
  c->total = 0;
}

static void sha512_update(sha512_ctx* c, const uint8_t* p, size_t n) {
  c->total += n;
  while (n) {
    size_t take = 128 - c->fill;
    if (take > n) take = n;
    memcpy(c->buf + c->fill, p, take);
    c->fill += take;
    p += take;
    n -= take;
    if (c->fill == 128) {
      sha512_block(c->h, c->buf);
      c->fill = 0;
    }
  }
}

static void sha512_final(sha512_ctx* c, uint8_t out[64]) {
  uint64_t bits = c->total * 8;
  uint8_t pad = 0x80;
  sha512_update(c, &pad, 1);
  uint8_t z = 0;
  while (c->fill != 112) sha512_update(c, &z, 1);
  uint8_t len[16] = {0};
  for (int i = 0; i < 8; ++i) len[15 - i] = (uint8_t)(bits >> (8 * i));
  sha512_update(c, len, 16);
  for (int i = 0; i < 8; ++i)
    for (int b = 0; b < 8; ++b) out[8 * i + b] = (uint8_t)(c->h[i] >> (56 - 8 * b));
}

void oracle_sha512(const uint8_t* in, size_t len, uint8_t out[64]) {
  sha512_ctx c;
  sha512_init(&c);
  sha512_update(&c, in, len);
  sha512_final(&c, out);
}

/* --------------------------------------------------------- field GF(2^255-19) */
typedef struct { uint64_t v[5]; } fe;
static const uint64_t MASK51 = (1ULL << 51) - 1;

static void fe_0(fe* r) { memset(r, 0, sizeof *r); }
static void fe_1(fe* r) { fe_0(r); r->v[0] = 1; }

/* loads the low 255 bits; values >= p are kept as-is (dalek FieldElement::from_bytes) */
static void fe_from_bytes(fe* r, const uint8_t b[32]) {
  uint64_t w[4];
  for (int i = 0; i < 4; ++i) {
    uint64_t v = 0;
    for (int j = 7; j >= 0; --j) v = (v << 8) | b[8 * i + j];
    w[i] = v;
  }
  r->v[0] = w[0] & MASK51;
  r->v[1] = ((w[0] >> 51) | (w[1] << 13)) & MASK51;
  r->v[2] = ((w[1] >> 38) | (w[2] << 26)) & MASK51;
  r->v[3] = ((w[2] >> 25) | (w[3] << 39)) & MASK51;
  r->v[4] = (w[3] >> 12) & MASK51;
}

static void fe_carry(fe* r) {
  for (int pass = 0; pass < 2; ++pass) {
    uint64_t c;
    c = r->v[0] >> 51; r->v[0] &= MASK51; r->v[1] += c;
    c = r->v[1] >> 51; r->v[1] &= MASK51; r->v[2] += c;
    c = r->v[2] >> 51; r->v[2] &= MASK51; r->v[3] += c;
    c = r->v[3] >> 51; r->v[3] &= MASK51; r->v[4] += c;
    c = r->v[4] >> 51; r->v[4] &= MASK51; r->v[0] += 19 * c;
  }
}

/* canonical little-endian encoding (value fully reduced mod p) */
static void fe_to_bytes(uint8_t out[32], const fe* a) {
  fe t = *a;
  fe_carry(&t);
  /* now t < 2^255 + small; t >= p  <=>  t + 19 >= 2^255 */
  uint64_t q = (t.v[0] + 19) >> 51;
  q = (t.v[1] + q) >> 51;
  q = (t.v[2] + q) >> 51;
  q = (t.v[3] + q) >> 51;
  q = (t.v[4] + q) >> 51;
  t.v[0] += 19 * q;
  uint64_t c;
  c = t.v[0] >> 51; t.v[0] &= MASK51; t.v[1] += c;
  c = t.v[1] >> 51; t.v[1] &= MASK51; t.v[2] += c;
  c = t.v[2] >> 51; t.v[2] &= MASK51; t.v[3] += c;
  c = t.v[3] >> 51; t.v[3] &= MASK51; t.v[4] += c;
  t.v[4] &= MASK51;
  uint64_t w0 = t.v[0] | (t.v[1] << 51);
  uint64_t w1 = (t.v[1] >> 13) | (t.v[2] << 38);
  uint64_t w2 = (t.v[2] >> 26) | (t.v[3] << 25);
  uint64_t w3 = (t.v[3] >> 39) | (t.v[4] << 12);
  uint64_t w[4] = {w0, w1, w2, w3};
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 8; ++j) out[8 * i + j] = (uint8_t)(w[i] >> (8 * j));
}

static void fe_add(fe* r, const fe* a, const fe* b) {
  for (int i = 0; i < 5; ++i) r->v[i] = a->v[i] + b->v[i];
  fe_carry(r);
}

/* a - b computed as a + 16p - b (no underflow for carried inputs), then carried */
static void fe_sub(fe* r, const fe* a, const fe* b) {
  static const uint64_t P16[5] = {16 * ((1ULL << 51) - 19), 16 * MASK51, 16 * MASK51, 16 * MASK51, 16 * MASK51};
  for (int i = 0; i < 5; ++i) r->v[i] = a->v[i] + P16[i] - b->v[i];
  fe_carry(r);
}

static void fe_neg(fe* r, const fe* a) {
  fe z;
  fe_0(&z);
  fe_sub(r, &z, a);
}

static void fe_mul(fe* r, const fe* a, const fe* b) {
  const uint64_t *x = a->v, *y = b->v;
  uint64_t y19[5];
  for (int i = 0; i < 5; ++i) y19[i] = 19 * y[i];
  u128 t[5];
  t[0] = (u128)x[0] * y[0] + (u128)x[1] * y19[4] + (u128)x[2] * y19[3] + (u128)x[3] * y19[2] + (u128)x[4] * y19[1];
  t[1] = (u128)x[0] * y[1] + (u128)x[1] * y[0] + (u128)x[2] * y19[4] + (u128)x[3] * y19[3] + (u128)x[4] * y19[2];
  t[2] = (u128)x[0] * y[2] + (u128)x[1] * y[1] + (u128)x[2] * y[0] + (u128)x[3] * y19[4] + (u128)x[4] * y19[3];
  t[3] = (u128)x[0] * y[3] + (u128)x[1] * y[2] + (u128)x[2] * y[1] + (u128)x[3] * y[0] + (u128)x[4] * y19[4];
  t[4] = (u128)x[0] * y[4] + (u128)x[1] * y[3] + (u128)x[2] * y[2] + (u128)x[3] * y[1] + (u128)x[4] * y[0];
  for (int i = 0; i < 4; ++i) {
    t[i + 1] += (uint64_t)(t[i] >> 51);
    t[i] &= MASK51;
  }
  uint64_t c = (uint64_t)(t[4] >> 51);
  t[4] &= MASK51;
  for (int i = 0; i < 5; ++i) r->v[i] = (uint64_t)t[i];
  r->v[0] += 19 * c;
  fe_carry(r);
}

static void fe_sq(fe* r, const fe* a) { fe_mul(r, a, a); }

static void fe_sqn(fe* r, const fe* a, int n) {
  *r = *a;
  for (int i = 0; i < n; ++i) fe_sq(r, r);
}

/* returns z^(2^250 - 1) and z^11 (shared prefix of pow22523 and invert) */
static void fe_pow_chain(fe* z250, fe* z11, const fe* z) {
  fe z2, z8, z9, z22, z5, z10, z20, z40, z50, z100, z200, t;
  fe_sq(&z2, z);            /* 2 */
  fe_sqn(&z8, &z2, 2);      /* 8 */
  fe_mul(&z9, &z8, z);      /* 9 */
  fe_mul(z11, &z9, &z2);    /* 11 */
  fe_sq(&z22, z11);         /* 22 */
  fe_mul(&z5, &z22, &z9);   /* 31 = 2^5 - 1 */
  fe_sqn(&t, &z5, 5);
  fe_mul(&z10, &t, &z5);    /* 2^10 - 1 */
  fe_sqn(&t, &z10, 10);
  fe_mul(&z20, &t, &z10);   /* 2^20 - 1 */
  fe_sqn(&t, &z20, 20);
  fe_mul(&z40, &t, &z20);   /* 2^40 - 1 */
  fe_sqn(&t, &z40, 10);
  fe_mul(&z50, &t, &z10);   /* 2^50 - 1 */
  fe_sqn(&t, &z50, 50);
  fe_mul(&z100, &t, &z50);  /* 2^100 - 1 */
  fe_sqn(&t, &z100, 100);
  fe_mul(&z200, &t, &z100); /* 2^200 - 1 */
  fe_sqn(&t, &z200, 50);
  fe_mul(z250, &t, &z50);   /* 2^250 - 1 */
}

static void fe_invert(fe* r, const fe* z) { /* z^(p-2) = z^(2^255 - 21) */
  fe z250, z11, t;
  fe_pow_chain(&z250, &z11, z);
  fe_sqn(&t, &z250, 5);
  fe_mul(r, &t, &z11);
}

static void fe_pow22523(fe* r, const fe* z) { /* z^((p-5)/8) = z^(2^252 - 3) */
  fe z250, z11, t;
  fe_pow_chain(&z250, &z11, z);
  fe_sqn(&t, &z250, 2);
  fe_mul(r, &t, z);
}

static int fe_eq(const fe* a, const fe* b) {
  uint8_t x[32], y[32];
  fe_to_bytes(x, a);
  fe_to_bytes(y, b);
  return memcmp(x, y, 32) == 0;
}

static int fe_is_negative(const fe* a) {
  uint8_t x[32];
  fe_to_bytes(x, a);
  return x[0] & 1;
}

static fe FE_D, FE_D2, FE_SQRTM1;

/* ------------------------------------------------------------- group (extended) */
typedef struct { fe X, Y, Z, T; } ge;

static void ge_identity(ge* p) {
  fe_0(&p->X);
  fe_1(&p->Y);
  fe_1(&p->Z);
  fe_0(&p->T);
}

/* unified addition, a = -1, complete (Hisil–Wong–Carter–Dawson 2008 §3.1) */
static void ge_add(ge* r, const ge* p, const ge* q) {
  fe a, b, c, d, e, f, g, h, t0, t1;
  fe_sub(&t0, &p->Y, &p->X);
  fe_sub(&t1, &q->Y, &q->X);
  fe_mul(&a, &t0, &t1);
  fe_add(&t0, &p->Y, &p->X);
  fe_add(&t1, &q->Y, &q->X);
  fe_mul(&b, &t0, &t1);
  fe_mul(&c, &p->T, &q->T);
  fe_mul(&c, &c, &FE_D2);
  fe_mul(&d, &p->Z, &q->Z);
  fe_add(&d, &d, &d);
  fe_sub(&e, &b, &a);
  fe_sub(&f, &d, &c);
  fe_add(&g, &d, &c);
  fe_add(&h, &b, &a);
  fe_mul(&r->X, &e, &f);
  fe_mul(&r->Y, &g, &h);
  fe_mul(&r->T, &e, &h);
  fe_mul(&r->Z, &f, &g);
}

static void ge_neg(ge* r, const ge* p) {
  fe_neg(&r->X, &p->X);
  r->Y = p->Y;
  r->Z = p->Z;
  fe_neg(&r->T, &p->T);
}

/* dedicated doubling, a = -1 (dbl-2008-hwcd) */
static void ge_dbl(ge* r, const ge* p) {
  fe a, b, c, e, g, f, h, t;
  fe_sq(&a, &p->X);
  fe_sq(&b, &p->Y);
  fe_sq(&c, &p->Z);
  fe_add(&c, &c, &c);
  fe_add(&t, &p->X, &p->Y);
  fe_sq(&e, &t);
  fe_sub(&e, &e, &a);
  fe_sub(&e, &e, &b);      /* E = 2XY */
  fe_sub(&g, &b, &a);      /* G = -A + B */
  fe_sub(&f, &g, &c);      /* F = G - C */
  fe_neg(&h, &a);
  fe_sub(&h, &h, &b);      /* H = -A - B */
  fe_mul(&r->X, &e, &f);
  fe_mul(&r->Y, &g, &h);
  fe_mul(&r->T, &e, &h);
  fe_mul(&r->Z, &f, &g);
}

static void ge_to_bytes(uint8_t out[32], const ge* p) {
  fe zi, x, y;
  fe_invert(&zi, &p->Z);
  fe_mul(&x, &p->X, &zi);
  fe_mul(&y, &p->Y, &zi);
  fe_to_bytes(out, &y);
  out[31] ^= (uint8_t)(fe_is_negative(&x) << 7);
}

/* sqrt_ratio_i(u, v): (1, +sqrt(u/v)) if u/v square, (1, 0) if u = 0, (0, *) otherwise;
 * also (0, sqrt(i*u/v)) for non-squares — only the flag matters for decompression. */
static int fe_sqrt_ratio_i(fe* r, const fe* u, const fe* v) {
  fe v3, v7, t, chk, nu, nui, rp;
  fe_sq(&v3, v);
  fe_mul(&v3, &v3, v);       /* v^3 */
  fe_sq(&v7, &v3);
  fe_mul(&v7, &v7, v);       /* v^7 */
  fe_mul(&t, u, &v7);
  fe_pow22523(&t, &t);       /* (u v^7)^((p-5)/8) */
  fe_mul(&t, &t, &v3);
  fe_mul(r, &t, u);          /* r = u v^3 (u v^7)^((p-5)/8) */
  fe_sq(&chk, r);
  fe_mul(&chk, &chk, v);     /* v r^2 */
  fe_neg(&nu, u);
  fe_mul(&nui, &nu, &FE_SQRTM1);
  int correct = fe_eq(&chk, u);
  int flipped = fe_eq(&chk, &nu);
  int flipped_i = fe_eq(&chk, &nui);
  if (flipped || flipped_i) {
    fe_mul(&rp, r, &FE_SQRTM1);
    *r = rp;
  }
  if (fe_is_negative(r)) fe_neg(r, r);
  return correct || flipped;
}

/* dalek CompressedEdwardsY::decompress semantics (Appendix A V2) */
static int ge_from_bytes(ge* p, const uint8_t s[32]) {
  fe one, yy, u, v;
  fe_1(&one);
  fe_from_bytes(&p->Y, s);
  fe_1(&p->Z);
  fe_sq(&yy, &p->Y);
  fe_sub(&u, &yy, &one);
  fe_mul(&v, &yy, &FE_D);
  fe_add(&v, &v, &one);
  if (!fe_sqrt_ratio_i(&p->X, &u, &v)) return 0;
  if (s[31] >> 7) fe_neg(&p->X, &p->X);
  fe_mul(&p->T, &p->X, &p->Y);
  return 1;
}

/* ------------------------------------------------------------- scalars mod l */
static const uint64_t L64[4] = {0x5812631a5cf5d3edULL, 0x14def9dea2f79cd6ULL, 0, 0x1000000000000000ULL};

static void sc_load(uint64_t w[4], const uint8_t b[32]) {
  for (int i = 0; i < 4; ++i) {
    uint64_t v = 0;
    for (int j = 7; j >= 0; --j) v = (v << 8) | b[8 * i + j];
    w[i] = v;
  }
}

static void sc_store(uint8_t b[32], const uint64_t w[4]) {
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 8; ++j) b[8 * i + j] = (uint8_t)(w[i] >> (8 * j));
}

static int sc_geq_l(const uint64_t w[4]) {
  for (int i = 3; i >= 0; --i) {
    if (w[i] > L64[i]) return 1;
    if (w[i] < L64[i]) return 0;
  }
  return 1;
}

static void sc_sub_l(uint64_t w[4]) {
  uint64_t borrow = 0;
  for (int i = 0; i < 4; ++i) {
    u128 d = (u128)w[i] - L64[i] - borrow;
    w[i] = (uint64_t)d;
    borrow = (uint64_t)(d >> 127);
  }
}

/* x (little-endian, nbytes) mod l — bit-serial reduction, most significant bit first:
 * r <- 2r + bit; if r >= l: r -= l. Invariant r < l < 2^253, so 2r+1 < 2^254 fits. */
static void sc_reduce_bytes(uint64_t r[4], const uint8_t* x, size_t nbytes) {
  r[0] = r[1] = r[2] = r[3] = 0;
  for (size_t bi = nbytes * 8; bi-- > 0;) {
    int bit = (x[bi >> 3] >> (bi & 7)) & 1;
    r[3] = (r[3] << 1) | (r[2] >> 63);
    r[2] = (r[2] << 1) | (r[1] >> 63);
    r[1] = (r[1] << 1) | (r[0] >> 63);
    r[0] = (r[0] << 1) | (uint64_t)bit;
    if (sc_geq_l(r)) sc_sub_l(r);
  }
}

void oracle_sc_reduce64(const uint8_t in[64], uint8_t out[32]) {
  uint64_t r[4];
  sc_reduce_bytes(r, in, 64);
  sc_store(out, r);
}

int oracle_sc_is_canonical(const uint8_t s[32]) {
  uint64_t w[4];
  sc_load(w, s);
  return !sc_geq_l(w);
}

void oracle_sc_muladd(const uint8_t a[32], const uint8_t b[32], const uint8_t c[32], uint8_t out[32]) {
  uint64_t x[4], y[4], z[4], prod[8] = {0};
  sc_load(x, a);
  sc_load(y, b);
  sc_load(z, c);
  for (int i = 0; i < 4; ++i) {
    u128 carry = 0;
    for (int j = 0; j < 4; ++j) {
      u128 t = (u128)x[i] * y[j] + prod[i + j] + carry;
      prod[i + j] = (uint64_t)t;
      carry = t >> 64;
    }
    prod[i + 4] = (uint64_t)carry;
  }
  u128 carry = 0;
  for (int i = 0; i < 8; ++i) {
    u128 t = (u128)prod[i] + (i < 4 ? z[i] : 0) + carry;
    prod[i] = (uint64_t)t;
    carry = t >> 64;
  }
  uint8_t bytes[72] = {0};
  for (int i = 0; i < 8; ++i)
    for (int j = 0; j < 8; ++j) bytes[8 * i + j] = (uint8_t)(prod[i] >> (8 * j));
  bytes[64] = (uint8_t)carry;
  uint64_t r[4];
  sc_reduce_bytes(r, bytes, 65);
  sc_store(out, r);
}

/* width-w non-adjacent form of a scalar < 2^253 (digits odd, |d| < 2^(w-1)) */
static void sc_naf(int8_t naf[256], const uint8_t s[32], int w) {
  uint64_t x[5];
  sc_load(x, s);
  x[4] = 0;
  memset(naf, 0, 256);
  const uint64_t width = 1ULL << w, mask = width - 1;
  uint64_t carry = 0;
  int pos = 0;
  while (pos < 256) {
    int idx = pos / 64, bit = pos % 64;
    uint64_t buf = (bit < 64 - w) ? (x[idx] >> bit) : ((x[idx] >> bit) | (x[idx + 1] << (64 - bit)));
    uint64_t window = carry + (buf & mask);
    if ((window & 1) == 0) {
      pos += 1;
      continue;
    }
    if (window < width / 2) {
      carry = 0;
      naf[pos] = (int8_t)window;
    } else {
      carry = 1;
      naf[pos] = (int8_t)((int64_t)window - (int64_t)width);
    }
    pos += w;
  }
}

/* ------------------------------------------------------------- constants/init */
static ge GE_B;
static ge B_ODD[64]; /* (2i+1) B, i = 0..63, for NAF-8 */
static pthread_once_t init_once = PTHREAD_ONCE_INIT;

static void fe_from_u64(fe* r, uint64_t x) {
  fe_0(r);
  r->v[0] = x & MASK51;
  r->v[1] = x >> 51;
}

static void oracle_init_impl(void) {
  fe n, dn, t;
  /* d = -121665 / 121666 */
  fe_from_u64(&n, 121665);
  fe_neg(&n, &n);
  fe_from_u64(&dn, 121666);
  fe_invert(&t, &dn);
  fe_mul(&FE_D, &n, &t);
  fe_add(&FE_D2, &FE_D, &FE_D);
  /* sqrt(-1) = 2^((p-1)/4); (p-1)/4 = 2^253 - 5: computed as 2^(2^253-5) by square-and-multiply */
  fe two, acc;
  fe_from_u64(&two, 2);
  fe_1(&acc);
  /* exponent bits: 2^253 - 5 = 0b1...1011 (253 bits: bit2 = 0, others set) */
  for (int bit = 252; bit >= 0; --bit) {
    fe_sq(&acc, &acc);
    if (bit != 2) fe_mul(&acc, &acc, &two);
  }
  FE_SQRTM1 = acc;
  /* base point: y = 4/5, x even */
  fe four, five, y;
  uint8_t enc[32];
  fe_from_u64(&four, 4);
  fe_from_u64(&five, 5);
  fe_invert(&t, &five);
  fe_mul(&y, &four, &t);
  fe_to_bytes(enc, &y);
  ge_from_bytes(&GE_B, enc);
  ge b2;
  ge_dbl(&b2, &GE_B);
  B_ODD[0] = GE_B;
  for (int i = 1; i < 64; ++i) ge_add(&B_ODD[i], &B_ODD[i - 1], &b2);
}

static void oracle_init(void) { pthread_once(&init_once, oracle_init_impl); }

/* R = [a]A + [b]B, vartime, NAF-5 on A and NAF-8 on B (dalek vartime_double_scalar_mul_basepoint shape) */
static void ge_double_scalarmult_vartime(ge* r, const uint8_t a[32], const ge* A, const uint8_t b[32]) {
  int8_t an[256], bn[256];
  sc_naf(an, a, 5);
  sc_naf(bn, b, 8);
  ge tA[8], A2; /* (2i+1) A */
  tA[0] = *A;
  ge_dbl(&A2, A);
  for (int i = 1; i < 8; ++i) ge_add(&tA[i], &tA[i - 1], &A2);
  int i = 255;
  while (i >= 0 && an[i] == 0 && bn[i] == 0) --i;
  ge acc;
  ge_identity(&acc);
  for (; i >= 0; --i) {
    ge t;
    ge_dbl(&t, &acc);
    acc = t;
    if (an[i] > 0) {
      ge_add(&t, &acc, &tA[an[i] / 2]);
      acc = t;
    } else if (an[i] < 0) {
      ge neg;
      ge_neg(&neg, &tA[(-an[i]) / 2]);
      ge_add(&t, &acc, &neg);
      acc = t;
    }
    if (bn[i] > 0) {
      ge_add(&t, &acc, &B_ODD[bn[i] / 2]);
      acc = t;
    } else if (bn[i] < 0) {
      ge neg;
      ge_neg(&neg, &B_ODD[(-bn[i]) / 2]);
      ge_add(&t, &acc, &neg);
      acc = t;
    }
  }
  *r = acc;
}

/* plain MSB-first double-and-add over all 256 bits (any scalar, any point) */
static void ge_scalarmult(ge* r, const uint8_t s[32], const ge* p) {
  ge acc, t;
  ge_identity(&acc);
  for (int bi = 255; bi >= 0; --bi) {
    ge_dbl(&t, &acc);
    acc = t;
    if ((s[bi >> 3] >> (bi & 7)) & 1) {
      ge_add(&t, &acc, p);
      acc = t;
    }
  }
  *r = acc;
}

/* ---------------------------------------------------------------- policies */
/* libsodium 1.0.18 ge25519_is_canonical: y-encoding (sign bit ignored) < p */
static int enc_y_canonical(const uint8_t s[32]) {
  /* y >= p iff bytes 1..30 are 0xff, byte31&0x7f == 0x7f and byte0 >= 0xed */
  if ((s[31] & 0x7f) != 0x7f) return 1;
  for (int i = 30; i >= 1; --i)
    if (s[i] != 0xff) return 1;
  return s[0] < 0xed;
}

/* libsodium 1.0.18 ge25519_has_small_order: y (sign bit masked) in the 7-entry blocklist
 * {0, 1, y8a, y8b, p-1, p, p+1}. The order-8 y values are computed at first use. */
static uint8_t SMALL_Y[7][32];
static pthread_once_t small_once = PTHREAD_ONCE_INIT;
static void ge_scalarmult(ge* r, const uint8_t s[32], const ge* p);
static void small_init(void) {
  oracle_init();
  memset(SMALL_Y, 0, sizeof SMALL_Y);
  /* Find T8 of exact order 8 as [l]P for a curve point P with a torsion component, then
   * the y's of the small-order points are y([j]T8), j = 0..4: {1, y8a, 0, y8b, -1}. */
  uint8_t lbytes[32];
  sc_store(lbytes, L64);
  ge T8;
  int have = 0;
  for (uint8_t yv = 2; yv < 255 && !have; ++yv) {
    uint8_t enc[32] = {0};
    enc[0] = yv;
    ge P, Q, D;
    if (!ge_from_bytes(&P, enc)) continue;
    ge_scalarmult(&Q, lbytes, &P);
    ge_dbl(&D, &Q);
    ge_dbl(&D, &D);
    uint8_t e4[32];
    ge_to_bytes(e4, &D);
    static const uint8_t ident[32] = {1};
    if (memcmp(e4, ident, 32) != 0) { /* [4]Q != identity  =>  Q has order 8 */
      T8 = Q;
      have = 1;
    }
  }
  ge acc = T8;
  for (int j = 1; j <= 4; ++j) {
    uint8_t e[32];
    ge_to_bytes(e, &acc);
    e[31] &= 0x7f;
    memcpy(SMALL_Y[j - 1], e, 32); /* j=1: y8a, 2: 0, 3: y8b, 4: p-1 */
    ge t;
    ge_add(&t, &acc, &T8);
    acc = t;
  }
  memset(SMALL_Y[4], 0, 32);
  SMALL_Y[4][0] = 1; /* identity */
  /* non-canonical aliases p and p+1 of y = 0 and y = 1 */
  for (int k = 5; k < 7; ++k) {
    memset(SMALL_Y[k], 0xff, 32);
    SMALL_Y[k][31] = 0x7f;
  }
  SMALL_Y[5][0] = 0xed;
  SMALL_Y[6][0] = 0xee;
}

static int enc_small_order(const uint8_t s[32]) {
  pthread_once(&small_once, small_init);
  uint8_t m[32];
  memcpy(m, s, 32);
  m[31] &= 0x7f;
  for (int k = 0; k < 7; ++k)
    if (memcmp(m, SMALL_Y[k], 32) == 0) return 1;
  return 0;
}

/* ------------------------------------------------------------------ verify */
int oracle_verify(const uint8_t pk[32], const uint8_t sig[64], const uint8_t* msg, size_t len, int policy) {
  oracle_init();
  const uint8_t* Rb = sig;
  const uint8_t* Sb = sig + 32;
  /* V1 */
  if (!oracle_sc_is_canonical(Sb)) return 0;
  if (policy == ORACLE_POLICY_LIBSODIUM_1_0_18) {
    if (enc_small_order(Rb)) return 0;
    if (!enc_y_canonical(pk) || enc_small_order(pk)) return 0;
  }
  /* V2 */
  ge A;
  if (!ge_from_bytes(&A, pk)) return 0;
  /* V3 */
  sha512_ctx c;
  uint8_t h[64], k[32];
  sha512_init(&c);
  sha512_update(&c, Rb, 32);
  sha512_update(&c, pk, 32);
  sha512_update(&c, msg, len);
  sha512_final(&c, h);
  oracle_sc_reduce64(h, k);
  /* V4 */
  ge negA, Rp;
  ge_neg(&negA, &A);
  ge_double_scalarmult_vartime(&Rp, k, &negA, Sb);
  /* V5, V6 */
  uint8_t enc[32];
  ge_to_bytes(enc, &Rp);
  return memcmp(enc, Rb, 32) == 0;
}

typedef struct {
  const uint8_t *pk, *sig, *msg;
  const uint32_t* off;
  size_t lo, hi;
  int policy;
  uint8_t* ok;
} batch_job;

static void* batch_worker(void* p) {
  batch_job* j = (batch_job*)p;
  for (size_t i = j->lo; i < j->hi; ++i)
    j->ok[i] = (uint8_t)oracle_verify(j->pk + 32 * i, j->sig + 64 * i, j->msg + j->off[i], j->off[i + 1] - j->off[i],
                                      j->policy);
  return NULL;
}

void oracle_verify_batch(const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, const uint32_t* msg_off, size_t n,
                         int policy, uint32_t* verdicts, int threads) {
  oracle_init();
  if (threads <= 0) threads = 1;
  if ((size_t)threads > n && n > 0) threads = (int)n;
  uint8_t* ok = (uint8_t*)calloc(n ? n : 1, 1);
  pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
  batch_job* jobs = (batch_job*)calloc((size_t)threads, sizeof(batch_job));
  for (int t = 0; t < threads; ++t) {
    jobs[t] = (batch_job){pk, sig, msg, msg_off, n * (size_t)t / (size_t)threads, n * (size_t)(t + 1) / (size_t)threads,
                          policy, ok};
    if (threads == 1)
      batch_worker(&jobs[t]);
    else
      pthread_create(&th[t], NULL, batch_worker, &jobs[t]);
  }
  if (threads > 1)
    for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
  size_t words = (n + 31) / 32;
  memset(verdicts, 0, words * 4);
  for (size_t i = 0; i < n; ++i)
    if (ok[i]) verdicts[i / 32] |= 1u << (i % 32);
  free(ok);
  free(th);
  free(jobs);
}

/* ------------------------------------------------------------- signing (RFC 8032) */
static void expand_seed(const uint8_t seed[32], uint8_t a[32], uint8_t prefix[32]) {
  uint8_t h[64];
  oracle_sha512(seed, 32, h);
  h[0] &= 248;
  h[31] &= 127;
  h[31] |= 64;
  memcpy(a, h, 32);
  memcpy(prefix, h + 32, 32);
}

void oracle_public_key(const uint8_t seed[32], uint8_t pk[32]) {
  oracle_init();
  uint8_t a[32], prefix[32];
  expand_seed(seed, a, prefix);
  ge A;
  ge_scalarmult(&A, a, &GE_B);
  ge_to_bytes(pk, &A);
}

void oracle_sign(const uint8_t seed[32], const uint8_t* msg, size_t len, uint8_t sig[64]) {
  oracle_init();
  uint8_t a[32], prefix[32], pk[32], h[64], r[32], k[32];
  expand_seed(seed, a, prefix);
  ge A, R;
  ge_scalarmult(&A, a, &GE_B);
  ge_to_bytes(pk, &A);
  sha512_ctx c;
  sha512_init(&c);
  sha512_update(&c, prefix, 32);
  sha512_update(&c, msg, len);
  sha512_final(&c, h);
  oracle_sc_reduce64(h, r);
  ge_scalarmult(&R, r, &GE_B);
  ge_to_bytes(sig, &R);
  sha512_init(&c);
  sha512_update(&c, sig, 32);
  sha512_update(&c, pk, 32);
  sha512_update(&c, msg, len);
  sha512_final(&c, h);
  oracle_sc_reduce64(h, k);
  oracle_sc_muladd(k, a, r, sig + 32);
}

void oracle_scalarmult_base(const uint8_t s[32], uint8_t out[32]) {
  oracle_init();
  ge R;
  ge_scalarmult(&R, s, &GE_B);
  ge_to_bytes(out, &R);
}

int oracle_point_add(const uint8_t p[32], const uint8_t q[32], uint8_t out[32]) {
  oracle_init();
  ge P, Q, R;
  if (!ge_from_bytes(&P, p) || !ge_from_bytes(&Q, q)) return 0;
  ge_add(&R, &P, &Q);
  ge_to_bytes(out, &R);
  return 1;
}

int oracle_scalarmult(const uint8_t s[32], const uint8_t p[32], uint8_t out[32]) {
  oracle_init();
  ge P, R;
  if (!ge_from_bytes(&P, p)) return 0;
  ge_scalarmult(&R, s, &P);
  ge_to_bytes(out, &R);
  return 1;
}

int oracle_decompress_ok(const uint8_t p[32]) {
  oracle_init();
  ge P;
  return ge_from_bytes(&P, p);
}

/* ------------------------------------------------------------- generator */
static void put_u64le(uint8_t* p, uint64_t v) {
  for (int i = 0; i < 8; ++i) p[i] = (uint8_t)(v >> (8 * i));
}

void oracle_gen_seed(uint64_t cfg_seed, uint64_t i, uint8_t seed[32]) {
  uint8_t buf[9 + 16], h[64];
  memcpy(buf, "at2v/seed", 9);
  put_u64le(buf + 9, cfg_seed);
  put_u64le(buf + 17, i);
  oracle_sha512(buf, sizeof buf, h);
  memcpy(seed, h, 32);
}

void oracle_gen_msg(uint64_t cfg_seed, uint64_t i, uint8_t* msg, size_t msg_len) {
  uint8_t buf[8 + 24], h[64];
  memcpy(buf, "at2v/msg", 8);
  put_u64le(buf + 8, cfg_seed);
  put_u64le(buf + 16, i);
  size_t done = 0;
  for (uint64_t ctr = 0; done < msg_len; ++ctr) {
    put_u64le(buf + 24, ctr);
    oracle_sha512(buf, sizeof buf, h);
    size_t take = msg_len - done < 64 ? msg_len - done : 64;
    memcpy(msg + done, h, take);
    done += take;
  }
}

typedef struct {
  uint64_t cfg_seed, first;
  size_t lo, hi, msg_len;
  uint8_t *pk, *sig, *msg;
} gen_job;

static void* gen_worker(void* p) {
  gen_job* j = (gen_job*)p;
  for (size_t t = j->lo; t < j->hi; ++t) {
    uint8_t seed[32];
    oracle_gen_seed(j->cfg_seed, j->first + t, seed);
    uint8_t* m = j->msg + t * j->msg_len;
    oracle_gen_msg(j->cfg_seed, j->first + t, m, j->msg_len);
    oracle_public_key(seed, j->pk + 32 * t);
    oracle_sign(seed, m, j->msg_len, j->sig + 64 * t);
  }
  return NULL;
}

void oracle_gen_records(uint64_t cfg_seed, uint64_t first, size_t n, size_t msg_len, uint8_t* pk, uint8_t* sig,
                        uint8_t* msg, int threads) {
  oracle_init();
  if (threads <= 0) threads = 1;
  pthread_t th[256];
  gen_job jobs[256];
  if (threads > 256) threads = 256;
  for (int t = 0; t < threads; ++t) {
    jobs[t] = (gen_job){cfg_seed, first, n * (size_t)t / (size_t)threads, n * (size_t)(t + 1) / (size_t)threads,
                        msg_len, pk, sig, msg};
    pthread_create(&th[t], NULL, gen_worker, &jobs[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
}

size_t oracle_thin_transaction(const uint8_t recipient[32], uint64_t amount, uint8_t out[48]) {
  put_u64le(out, 32);
  memcpy(out + 8, recipient, 32);
  put_u64le(out + 40, amount);
  return 48;
}

/* ------------------------------------------------- AT2 config-1 transactions */
/* 64 senders x sequences 1..64; tx t = (seq-1)*64 + sender. Recipient = another sender's public key,
 * amount in [1, 1000], both from SHA-512("at2v/tx" || u64le(cfg_seed) || u64le(t)).
 * M = bincode(ThinTransaction{recipient, amount}) (src/lib.rs:14-22), signed by the sender as
 * src/client.rs:77-78 does. Outputs n = 4096 records with 48-byte messages plus (sender, sequence). */
void oracle_gen_at2_transactions(uint64_t cfg_seed, uint8_t* pk, uint8_t* sig, uint8_t* msg, uint32_t* sender,
                                 uint32_t* sequence) {
  oracle_init();
  uint8_t seeds[64][32], pks[64][32];
  for (int s = 0; s < 64; ++s) {
    oracle_gen_seed(cfg_seed, (uint64_t)s, seeds[s]);
    oracle_public_key(seeds[s], pks[s]);
  }
  for (uint32_t t = 0; t < 4096; ++t) {
    uint32_t s = t % 64, seq = t / 64 + 1;
    uint8_t buf[7 + 16], h[64];
    memcpy(buf, "at2v/tx", 7);
    put_u64le(buf + 7, cfg_seed);
    put_u64le(buf + 15, t);
    oracle_sha512(buf, sizeof buf, h);
    uint32_t rcpt = (s + 1 + h[0] % 63) % 64;
    uint64_t r = 0;
    for (int b = 0; b < 8; ++b) r |= (uint64_t)h[8 + b] << (8 * b);
    uint64_t amount = 1 + r % 1000;
    uint8_t* m = msg + 48 * (size_t)t;
    oracle_thin_transaction(pks[rcpt], amount, m);
    memcpy(pk + 32 * (size_t)t, pks[s], 32);
    oracle_sign(seeds[s], m, 48, sig + 64 * (size_t)t);
    sender[t] = s;
    sequence[t] = seq;
  }
}

/* --------------------------------------------------- adversarial generator */
/* sign with secret from seed but hash the given (possibly non-matching) public key bytes */
static void sign_with_pk(const uint8_t seed[32], const uint8_t pkb[32], const uint8_t* msg, size_t len, uint8_t sig[64]) {
  uint8_t a[32], prefix[32], h[64], r[32], k[32];
  expand_seed(seed, a, prefix);
  sha512_ctx c;
  sha512_init(&c);
  sha512_update(&c, prefix, 32);
  sha512_update(&c, msg, len);
  sha512_final(&c, h);
  oracle_sc_reduce64(h, r);
  ge R;
  ge_scalarmult(&R, r, &GE_B);
  ge_to_bytes(sig, &R);
  sha512_init(&c);
  sha512_update(&c, sig, 32);
  sha512_update(&c, pkb, 32);
  sha512_update(&c, msg, len);
  sha512_final(&c, h);
  oracle_sc_reduce64(h, k);
  oracle_sc_muladd(k, a, r, sig + 32);
}

/* the 14 encodings of small-order points: y in {1, p-1, 0, y8a, y8b, p, p+1} x sign bit */
void oracle_small_order_encoding(int idx, uint8_t out[32]) {
  pthread_once(&small_once, small_init);
  /* SMALL_Y: 0 y8a, 1 y=0, 2 y8b, 3 p-1, 4 one, 5 p, 6 p+1 */
  memcpy(out, SMALL_Y[(idx / 2) % 7], 32);
  if (idx & 1) out[31] |= 0x80;
}

static void add_l(uint8_t s[32]) { /* s += l (s < l so the result < 2^254) */
  uint64_t w[4];
  sc_load(w, s);
  u128 carry = 0;
  for (int i = 0; i < 4; ++i) {
    u128 t = (u128)w[i] + L64[i] + carry;
    w[i] = (uint64_t)t;
    carry = t >> 64;
  }
  sc_store(s, w);
}

typedef struct {
  uint64_t cfg_seed, first;
  size_t lo, hi, msg_len;
  uint8_t *pk, *sig, *msg, *cls;
} adv_job;

static void adv_one(uint64_t cfg_seed, uint64_t idx, size_t msg_len, uint8_t* pk, uint8_t* sig, uint8_t* m,
                    uint8_t* cls) {
  uint8_t seed[32], buf[8 + 16], h[64];
  oracle_gen_seed(cfg_seed, idx, seed);
  oracle_gen_msg(cfg_seed, idx, m, msg_len);
  memcpy(buf, "at2v/adv", 8);
  put_u64le(buf + 8, cfg_seed);
  put_u64le(buf + 16, idx);
  oracle_sha512(buf, sizeof buf, h);
  uint32_t u = ((uint32_t)h[0] | ((uint32_t)h[1] << 8)) % 1000;
  uint32_t v = (uint32_t)h[2] | ((uint32_t)h[3] << 8) | ((uint32_t)h[4] << 16);
  /* class thresholds (per mille): valid 900, sig-bitflip 40, msg-bitflip 10, S+l 15, S-top-bits 5,
   * non-canonical R 15, small-order A 10, A off-curve 5 */
  int c;
  if (u < 900) c = 0;
  else if (u < 940) c = 1;
  else if (u < 950) c = 2;
  else if (u < 965) c = 3;
  else if (u < 970) c = 4;
  else if (u < 985) c = 5;
  else if (u < 995) c = 6;
  else c = 7;
  *cls = (uint8_t)c;
  oracle_public_key(seed, pk);
  oracle_sign(seed, m, msg_len, sig);
  switch (c) {
    case 0: break;
    case 1: sig[(v >> 3) % 64] ^= (uint8_t)(1u << (v & 7)); break;
    case 2:
      if (msg_len) m[(v >> 3) % msg_len] ^= (uint8_t)(1u << (v & 7));
      else sig[0] ^= 1;
      break;
    case 3: add_l(sig + 32); break;
    case 4: sig[63] |= (uint8_t)(0x20u << (v % 3)); break;
    case 5: {
      int sub = v % 4;
      if (sub == 0) { /* y >= p encoding with random sign */
        memset(sig, 0xff, 32);
        sig[31] = 0x7f | (uint8_t)((v >> 2) & 0x80);
        sig[0] = (uint8_t)(0xed + (v >> 8) % 19);
      } else { /* would-accept-if-canonical: A = identity, S = 0, R' = identity; R = a non-canonical identity */
        memset(pk, 0, 32);
        pk[0] = 1;
        memset(sig + 32, 0, 32);
        memset(sig, 0, 32);
        if (sub == 1) { sig[0] = 1; sig[31] = 0x80; }                 /* x = 0 with sign bit */
        else if (sub == 2) { memset(sig, 0xff, 32); sig[0] = 0xee; sig[31] = 0x7f; } /* y = p + 1 */
        else { memset(sig, 0xff, 32); sig[0] = 0xee; sig[31] = 0xff; }              /* y = p + 1, sign bit */
      }
      break;
    }
    case 6: {
      int sub = v % 2;
      uint8_t T[32];
      oracle_small_order_encoding((int)((v >> 1) % 14), T);
      if (sub == 0) { /* A = small-order point; R = [S]B for random S  =>  accept iff [k]T == 0 */
        uint8_t S[32];
        memcpy(S, h + 8, 32);
        S[31] &= 0x0f; /* < 2^252 < l */
        memcpy(pk, T, 32);
        oracle_scalarmult_base(S, sig);
        memcpy(sig + 32, S, 32);
      } else { /* mixed order: A = A0 + T, signed with A0's secret; accept iff [k]T == 0 */
        uint8_t A0[32], Am[32];
        memcpy(A0, pk, 32);
        oracle_point_add(A0, T, Am);
        memcpy(pk, Am, 32);
        sign_with_pk(seed, pk, m, msg_len, sig);
      }
      break;
    }
    case 7: { /* A not on the curve: deterministic search over y for a failing decode */
      uint8_t cand[32];
      memcpy(cand, h + 8, 32);
      for (int tries = 0; tries < 256; ++tries) {
        if (!oracle_decompress_ok(cand)) break;
        cand[0] = (uint8_t)(cand[0] + 1);
      }
      memcpy(pk, cand, 32);
      break;
    }
  }
}

static void* adv_worker(void* p) {
  adv_job* j = (adv_job*)p;
  for (size_t t = j->lo; t < j->hi; ++t)
    adv_one(j->cfg_seed, j->first + t, j->msg_len, j->pk + 32 * t, j->sig + 64 * t, j->msg + t * j->msg_len,
            j->cls + t);
  return NULL;
}

void oracle_gen_adversarial(uint64_t cfg_seed, uint64_t first, size_t n, size_t msg_len, uint8_t* pk, uint8_t* sig,
                            uint8_t* msg, uint8_t* cls, int threads) {
  oracle_init();
  pthread_once(&small_once, small_init);
  if (threads <= 0) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t th[256];
  adv_job jobs[256];
  for (int t = 0; t < threads; ++t) {
    jobs[t] = (adv_job){cfg_seed, first, n * (size_t)t / (size_t)threads, n * (size_t)(t + 1) / (size_t)threads,
                        msg_len, pk, sig, msg, cls};
    pthread_create(&th[t], NULL, adv_worker, &jobs[t]);
  }
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
}
