// at2v_fe_base.h — GF(2^255-19) element, radix 2^25.5, 10 balanced signed int32 limbs.
//
// Compiles for gfx950 (hipcc) and for the host (g++: at2v_verify_one in at2v_cpu.cpp, and the CPU tests
// tests/test_host_core.py / test_verify_one_cpu.py). Design and bound proof: DESIGN.md §3, tools/gen_fe.py.
//
// Bound classes used by the curve formulas (at2v_ge.h):
//   carried  : |v_i| <= 2^(w_i-1) (+2^16 on limb 1)   — output of fe_mul/fe_sq/fe_carry32/fe_frombytes
//   k-term   : sum/difference of k carried elements    — fe_mul/fe_sq accept k <= 3
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define AT2V_HD __host__ __device__
#define AT2V_INLINE __forceinline__
#define AT2V_CONST_ARR __device__ const
#else
#define AT2V_HD
#define AT2V_INLINE inline __attribute__((always_inline))
#define AT2V_CONST_ARR static const
#endif
#define AT2V_CONST_FE constexpr fe

// 32x32 -> 64 signed multiply-add: one v_mad_i64_i32 on gfx950
#define AT2V_MAD(a, b, c) ((int64_t)(int32_t)(a) * (int64_t)(int32_t)(b) + (int64_t)(c))
#define AT2V_BIAS26 (1 << 25)
#define AT2V_BIAS25 (1 << 24)

#if defined(__HIP_DEVICE_COMPILE__)
// 2*x as a full-rate v_add_u32 (LLVM would emit the half-rate v_lshlrev_b32 on gfx950)
__device__ AT2V_INLINE int32_t at2v_dbl32(int32_t x) {
  int32_t r;
  asm("v_add_u32 %0, %1, %1" : "=v"(r) : "v"(x));
  return r;
}
#define AT2V_X2(x) at2v_dbl32(x)
#ifndef AT2V_FE_ASM_BLOCKS
// Column MADs as asm blocks (tools/gen_fe.py emit_block_asm): one v_mad_i64_i32 per column per block,
// the rounding bias as the SGPR addend of the first block. Plain C lets LLVM re-associate the bias
// out of the chains (10 extra 64-bit adds per multiply).
#define AT2V_FE_ASM_BLOCKS 1
#endif
#else
#define AT2V_X2(x) (2 * (x))
#undef AT2V_FE_ASM_BLOCKS
#define AT2V_FE_ASM_BLOCKS 0
#endif

namespace at2v {

struct fe {
  int32_t v[10];
};

AT2V_HD AT2V_INLINE void fe_0(fe& h) {
#pragma unroll
  for (int i = 0; i < 10; ++i) h.v[i] = 0;
}
AT2V_HD AT2V_INLINE void fe_1(fe& h) {
  fe_0(h);
  h.v[0] = 1;
}
AT2V_HD AT2V_INLINE void fe_add(fe& h, const fe& f, const fe& g) {
#pragma unroll
  for (int i = 0; i < 10; ++i) h.v[i] = f.v[i] + g.v[i];
}
AT2V_HD AT2V_INLINE void fe_sub(fe& h, const fe& f, const fe& g) {
#pragma unroll
  for (int i = 0; i < 10; ++i) h.v[i] = f.v[i] - g.v[i];
}
AT2V_HD AT2V_INLINE void fe_neg(fe& h, const fe& f) {
#pragma unroll
  for (int i = 0; i < 10; ++i) h.v[i] = -f.v[i];
}
// h = b ? g : f   (b is 0/1, per lane)
AT2V_HD AT2V_INLINE void fe_select(fe& h, const fe& f, const fe& g, int b) {
#pragma unroll
  for (int i = 0; i < 10; ++i) h.v[i] = b ? g.v[i] : f.v[i];
}

// Balanced floor-carry of the 10 biased column accumulators of a product (each column was
// initialised with its rounding bias 2^(w-1)): r_i = (h_i mod 2^w) - 2^(w-1), carry = h_i >> w.
// Two interleaved chains (critical path 7 carries instead of 11):
//   A: 0 -> 1 -> 2 -> 3 -> 4' -> 5          B: 4 -> 5 -> 6 -> 7 -> 8 -> 9 -> (x19) 0' -> 1
// Limb 4 is carried twice (its second pass re-adds the bias); limbs 1 and 5 end with a small spill
// (< 2^16), accounted for in tools/gen_fe.py carried_bound().
#define AT2V_EXT26(h) (((int32_t)(h) & 0x3ffffff) - (1 << 25))
#define AT2V_EXT25(h) (((int32_t)(h) & 0x1ffffff) - (1 << 24))
AT2V_HD AT2V_INLINE void fe_carry_wide(fe& r, int64_t h0, int64_t h1, int64_t h2, int64_t h3, int64_t h4, int64_t h5,
                                       int64_t h6, int64_t h7, int64_t h8, int64_t h9) {
  int64_t ca, cb;
  ca = h0 >> 26; h1 += ca; r.v[0] = AT2V_EXT26(h0);
  cb = h4 >> 26; h5 += cb; const int32_t t4 = AT2V_EXT26(h4);
  ca = h1 >> 25; h2 += ca; r.v[1] = AT2V_EXT25(h1);
  cb = h5 >> 25; h6 += cb; const int32_t t5 = AT2V_EXT25(h5);
  ca = h2 >> 26; h3 += ca; r.v[2] = AT2V_EXT26(h2);
  cb = h6 >> 26; h7 += cb; r.v[6] = AT2V_EXT26(h6);
  ca = h3 >> 25; r.v[3] = AT2V_EXT25(h3);
  const int64_t h4b = (int64_t)t4 + ca + (1 << 25);
  cb = h7 >> 25; h8 += cb; r.v[7] = AT2V_EXT25(h7);
  ca = h4b >> 26; r.v[5] = t5 + (int32_t)ca; r.v[4] = AT2V_EXT26(h4b);
  cb = h8 >> 26; h9 += cb; r.v[8] = AT2V_EXT26(h8);
  cb = h9 >> 25; r.v[9] = AT2V_EXT25(h9);
  const int64_t h0b = (int64_t)r.v[0] + cb * 19 + (1 << 25);
  cb = h0b >> 26;
  r.v[0] = AT2V_EXT26(h0b);
  r.v[1] += (int32_t)cb;
}

// Balanced carry of an element with int32 limbs (any |v_i| < 2^30): result is "carried".
AT2V_HD AT2V_INLINE void fe_carry32(fe& h) {
  int32_t c;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int w = (i & 1) ? 25 : 26;
    c = (h.v[i] + (1 << (w - 1))) >> w;
    h.v[i + 1] += c;
    h.v[i] -= c * (1 << w);
  }
  c = (h.v[9] + (1 << 24)) >> 25;
  h.v[9] -= c * (1 << 25);
  h.v[0] += 19 * c;
  c = (h.v[0] + (1 << 25)) >> 26;
  h.v[0] -= c * (1 << 26);
  h.v[1] += c;
}

// 32 little-endian bytes (given as 8 LE words) -> element. Bit 255 is ignored; values >= p are NOT
// reduced (dalek FieldElement::from_bytes semantics).
AT2V_HD AT2V_INLINE void fe_frombytes(fe& h, const uint32_t w[8]) {
  // bit offsets 0,26,51,77,102,128,153,179,204,230
  auto bits = [&](int off, int width) -> int32_t {
    const int k = off >> 5, s = off & 31;
    uint64_t v = (uint64_t)w[k] | ((k + 1 < 8) ? ((uint64_t)w[k + 1] << 32) : 0);
    return (int32_t)((v >> s) & ((1u << width) - 1));
  };
  h.v[0] = bits(0, 26);
  h.v[1] = bits(26, 25);
  h.v[2] = bits(51, 26);
  h.v[3] = bits(77, 25);
  h.v[4] = bits(102, 26);
  h.v[5] = bits(128, 25);
  h.v[6] = bits(153, 26);
  h.v[7] = bits(179, 25);
  h.v[8] = bits(204, 26);
  h.v[9] = bits(230, 25);
  fe_carry32(h);
}

// Canonical encoding (fully reduced mod p) as 8 little-endian words. Input: carried or k<=3-term.
AT2V_HD AT2V_INLINE void fe_tobytes(uint32_t out[8], const fe& f) {
  // add 4p limb-wise so every limb is positive, then three floor-carry passes
  int64_t t[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const int w = (i & 1) ? 25 : 26;
    int64_t p4 = (int64_t)4 * (((int64_t)1 << w) - 1);
    if (i == 0) p4 = (int64_t)4 * (((int64_t)1 << 26) - 19);
    t[i] = (int64_t)f.v[i] + p4;
  }
#pragma unroll
  for (int pass = 0; pass < 3; ++pass) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      const int w = (i & 1) ? 25 : 26;
      int64_t c = t[i] >> w;
      t[i] &= ((int64_t)1 << w) - 1;
      if (i < 9) t[i + 1] += c;
      else t[0] += 19 * c;
    }
  }
  // now 0 <= value < 2^255 with limbs in range; subtract p once if value >= p (value + 19 >= 2^255)
  int64_t q = (t[0] + 19) >> 26;
#pragma unroll
  for (int i = 1; i < 10; ++i) q = (t[i] + q) >> ((i & 1) ? 25 : 26);
  t[0] += 19 * q;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int w = (i & 1) ? 25 : 26;
    int64_t c = t[i] >> w;
    t[i] &= ((int64_t)1 << w) - 1;
    t[i + 1] += c;
  }
  t[9] &= ((int64_t)1 << 25) - 1;
  // pack 255 bits
  uint64_t acc = 0;
  int nb = 0, wi = 0;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const int w = (i & 1) ? 25 : 26;
    acc |= (uint64_t)t[i] << nb;
    nb += w;
    while (nb >= 32) {
      out[wi++] = (uint32_t)acc;
      acc >>= 32;
      nb -= 32;
    }
  }
  out[wi] = (uint32_t)acc;  // wi == 7, nb == 31
}

}  // namespace at2v
