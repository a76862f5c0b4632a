// at2v_sha512.h — SHA-512 (FIPS 180-4), one message per lane, for k = H(R || A || M) (SURVEY A V3)
// and for the deterministic record generator / signer kernels.
//
// 64-bit words on the 32-bit VALU: rotations as v_alignbit_b32 pairs, additions as v_lshl_add_u64. Rounds take the
// working variables in rotated order (no moves); the first 16 rounds are peeled, the other 64 run as a rolled loop of
// a 16-round body whose message schedule lives in a 16-entry circular register window.
#pragma once
#include "at2v_fe_base.h"

namespace at2v {

AT2V_CONST_ARR uint64_t SHA512_K[80] = {
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

AT2V_HD AT2V_INLINE uint64_t sha_ror(uint64_t x, int n) {
#if defined(__HIP_DEVICE_COMPILE__)
  // two v_alignbit_b32 (a 64-bit shift pair + OR would be four instructions)
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  uint32_t rlo, rhi;
  if (n < 32) {
    rlo = __builtin_amdgcn_alignbit(hi, lo, n);
    rhi = __builtin_amdgcn_alignbit(lo, hi, n);
  } else {
    rlo = __builtin_amdgcn_alignbit(lo, hi, n - 32);
    rhi = __builtin_amdgcn_alignbit(hi, lo, n - 32);
  }
  return ((uint64_t)rhi << 32) | rlo;
#else
  return (x >> n) | (x << (64 - n));
#endif
}
// x ^ y ^ z and maj(x, y, z) on 64-bit words; on gfx950 one v_bitop3_b32 per half (truth tables 0x96 and 0xe8,
// both symmetric in their operands) instead of two XORs, or an XOR and a bit-select. AT2V_SHA_BITOP3=0: plain C.
#ifndef AT2V_SHA_BITOP3
#define AT2V_SHA_BITOP3 1
#endif
#if defined(__HIP_DEVICE_COMPILE__) && AT2V_SHA_BITOP3
template <int LUT>
__device__ AT2V_INLINE uint64_t sha_bitop3(uint64_t x, uint64_t y, uint64_t z) {
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  u32x2 v;
  v.x = __builtin_amdgcn_bitop3_b32((uint32_t)x, (uint32_t)y, (uint32_t)z, LUT);
  v.y = __builtin_amdgcn_bitop3_b32((uint32_t)(x >> 32), (uint32_t)(y >> 32), (uint32_t)(z >> 32), LUT);
  // a bit cast of the pair, not (hi << 32) | lo: LLVM turns that disjoint OR into an ADD and splits the consuming
  // 64-bit adds into two zero-padded ones plus register moves
  return __builtin_bit_cast(uint64_t, v);
}
AT2V_HD AT2V_INLINE uint64_t sha_xor3(uint64_t x, uint64_t y, uint64_t z) { return sha_bitop3<0x96>(x, y, z); }
AT2V_HD AT2V_INLINE uint64_t sha_maj(uint64_t x, uint64_t y, uint64_t z) { return sha_bitop3<0xe8>(x, y, z); }
#else
AT2V_HD AT2V_INLINE uint64_t sha_xor3(uint64_t x, uint64_t y, uint64_t z) { return x ^ y ^ z; }
AT2V_HD AT2V_INLINE uint64_t sha_maj(uint64_t x, uint64_t y, uint64_t z) { return (x & y) ^ (z & (x ^ y)); }
#endif
// (hi << 32) | lo; on the device as a bit cast of the register pair (see sha_bitop3)
AT2V_HD AT2V_INLINE uint64_t sha_pair(uint32_t lo, uint32_t hi) {
#if defined(__HIP_DEVICE_COMPILE__)
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  u32x2 v;
  v.x = lo;
  v.y = hi;
  return __builtin_bit_cast(uint64_t, v);
#else
  return ((uint64_t)hi << 32) | lo;
#endif
}
AT2V_HD AT2V_INLINE uint32_t bswap32(uint32_t x) {
  return (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24);
}

AT2V_HD AT2V_INLINE void sha512_init(uint64_t h[8]) {
  h[0] = 0x6a09e667f3bcc908ULL; h[1] = 0xbb67ae8584caa73bULL; h[2] = 0x3c6ef372fe94f82bULL;
  h[3] = 0xa54ff53a5f1d36f1ULL; h[4] = 0x510e527fade682d1ULL; h[5] = 0x9b05688c2b3e6c1fULL;
  h[6] = 0x1f83d9abfb41bd6bULL; h[7] = 0x5be0cd19137e2179ULL;
}

// one round with the working variables passed in rotated order (no register moves between rounds)
AT2V_HD AT2V_INLINE void sha512_round(uint64_t a, uint64_t b, uint64_t c, uint64_t& d, uint64_t e, uint64_t f,
                                      uint64_t g, uint64_t& h, uint64_t kw) {
  const uint64_t S1 = sha_xor3(sha_ror(e, 14), sha_ror(e, 18), sha_ror(e, 41));
  const uint64_t ch = (e & f) ^ (~e & g);
  const uint64_t t1 = h + S1 + ch + kw;
  const uint64_t S0 = sha_xor3(sha_ror(a, 28), sha_ror(a, 34), sha_ror(a, 39));
  const uint64_t mj = sha_maj(a, b, c);
  d += t1;
  h = t1 + S0 + mj;
}

// 16 rounds r0 .. r0+15; SCHED: extend the message schedule in the 16-word circular window first
template <bool SCHED>
AT2V_HD AT2V_INLINE void sha512_rounds16(uint64_t s[8], uint64_t w[16], int r0) {
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    if (SCHED) {
      const uint64_t w15 = w[(i + 1) & 15], w2 = w[(i + 14) & 15];
      const uint64_t s0 = sha_xor3(sha_ror(w15, 1), sha_ror(w15, 8), w15 >> 7);
      const uint64_t s1 = sha_xor3(sha_ror(w2, 19), sha_ror(w2, 61), w2 >> 6);
      w[i] += s0 + w[(i + 9) & 15] + s1;
    }
    const uint64_t kw = SHA512_K[r0 + i] + w[i];
    // working variable j of round i is s[(j - i) mod 8] (a = s[0] in round 0)
    sha512_round(s[(8 - i % 8) % 8], s[(9 - i % 8) % 8], s[(10 - i % 8) % 8], s[(11 - i % 8) % 8],
                 s[(12 - i % 8) % 8], s[(13 - i % 8) % 8], s[(14 - i % 8) % 8], s[(15 - i % 8) % 8], kw);
  }
}

// one compression; w[16] = the block as big-endian 64-bit words (clobbered). The first 16 rounds use the block as
// is; the other 64 run as a rolled loop of a 16-round body (a multiple of 8 rounds: the rotated names line up).
AT2V_HD AT2V_INLINE void sha512_compress(uint64_t h[8], uint64_t w[16]) {
  uint64_t s[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) s[i] = h[i];
  sha512_rounds16<false>(s, w, 0);
#pragma unroll 1
  for (int r = 16; r < 80; r += 16) sha512_rounds16<true>(s, w, r);
#pragma unroll
  for (int i = 0; i < 8; ++i) h[i] += s[i];
}

// digest -> 16 little-endian 32-bit words of the 64-byte output (as bytes: big-endian h[0..7])
AT2V_HD AT2V_INLINE void sha512_digest_words(uint32_t out[16], const uint64_t h[8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    out[2 * i] = bswap32((uint32_t)(h[i] >> 32));
    out[2 * i + 1] = bswap32((uint32_t)h[i]);
  }
}

// SHA-512 of (prefix || M) where prefix is np 32-byte-word chunks given as LE words (np*8 words,
// np in {0,1,2}) and M is read through `msgword(j)` = the j-th little-endian 32-bit word of M
// (bytes 4j..4j+3; bytes past len may be garbage — they are masked here). msgword is called for every word of every
// block, with j clamped to len/4. len < 2^32.
template <int NPW, class MsgWord>
AT2V_HD AT2V_INLINE void sha512_prefixed(uint64_t h[8], const uint32_t* prefix, uint32_t len, MsgWord msgword) {
  sha512_init(h);
  const uint32_t total = (uint32_t)(4 * NPW) + len;                 // bytes hashed
  const uint32_t nblocks = (total + 17 + 127) >> 7;
  for (uint32_t b = 0; b < nblocks; ++b) {
    uint64_t w[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      uint32_t be[2];
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const uint32_t pos = (b << 7) + 8 * t + 4 * half;  // stream byte position (4-aligned)
        uint32_t le;
        // the prefix (<= 64 bytes) lives in block 0 only: static register index, no scratch
        if (2 * t + half < NPW && b == 0) {
          le = prefix[(2 * t + half) < NPW ? (2 * t + half) : 0];
        } else {
          const uint32_t mo = pos - 4 * NPW;                 // message byte offset
          // every lane reads a word (bytes past len are masked below): no divergent branch per word
          uint32_t v = msgword((mo < len ? mo : len) >> 2);
          const uint32_t nvalid = mo >= len ? 0u : (len - mo >= 4 ? 4u : len - mo);
          if (nvalid < 4) {
            v = nvalid ? (v & ((1u << (8 * nvalid)) - 1)) : 0u;
            if (mo <= len) v |= 0x80u << (8 * nvalid);        // the 0x80 pad byte lands at mo + nvalid == len
          }
          le = v;
        }
        be[half] = bswap32(le);
      }
      w[t] = sha_pair(be[1], be[0]);
    }
    if (b == nblocks - 1) {
      w[14] = 0;
      w[15] = (uint64_t)total * 8;
    }
    sha512_compress(h, w);
  }
}

// A message source that chooses, once per wave, between an unguarded reader (every lane's message ends well before the
// buffer end) and a bounds-checked one. Each SHA-512 instantiation is then straight-line code whose message loads the
// compiler can issue back to back; a wave-uniform branch per word between the two readers kept every load behind its
// own s_waitcnt (one memory latency per message word, ~26 per signature at 100-byte messages).
struct MsgNoTouch {
  AT2V_HD AT2V_INLINE void operator()() const {}
};
template <class Fast, class Slow, class Touch = MsgNoTouch>
struct MsgSplit {
  int fast;
  Fast f;
  Slow s;
  Touch touch;  // called once before the hash: consumes the kernel's early loads of the message (AT2V_MSG_TOUCH)
};

template <int NPW, class MsgWord>
AT2V_HD AT2V_INLINE void sha512_msg(uint64_t h[8], const uint32_t* prefix, uint32_t len, MsgWord& m) {
  sha512_prefixed<NPW>(h, prefix, len, m);
}
template <int NPW, class Fast, class Slow, class Touch>
AT2V_HD AT2V_INLINE void sha512_msg(uint64_t h[8], const uint32_t* prefix, uint32_t len,
                                    MsgSplit<Fast, Slow, Touch>& m) {
  m.touch();
  if (m.fast)
    sha512_prefixed<NPW>(h, prefix, len, m.f);
  else
    sha512_prefixed<NPW>(h, prefix, len, m.s);
}

}  // namespace at2v
