// at2v_fu_base.h — GF(2^255-19) element with UNSIGNED limbs, radix 2^25.5 (tools/gen_fu.py).
//
// Compiles for gfx950 (hipcc) and for the host (g++). Limbs are non-negative; "carried" means limb i < 2^W[i]
// (limb 1 < 2^25 + kFuLimb1Spill). Subtractions add a multiple of p whose limbs dominate the subtrahend's.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#ifndef AT2V_HD
#define AT2V_HD __host__ __device__
#define AT2V_INLINE __forceinline__
#endif
#else
#ifndef AT2V_HD
#define AT2V_HD
#define AT2V_INLINE inline __attribute__((always_inline))
#endif
#endif

// 32x32 -> 64 unsigned multiply-add: one v_mad_u64_u32 on gfx950; small-constant scaling of a 32-bit operand
#if defined(AT2V_FU_CHECK) && !defined(__HIPCC__)
// TEST ONLY (tests/host/verify_host.cpp built with -DAT2V_FU_CHECK): every scaled operand must fit 32 bits and every
// column sum 64 bits; a violation of the bounds tools/gen_fu.py proves aborts
#include <cstdio>
#include <cstdlib>
inline uint32_t at2v_usc_checked(uint64_t s, uint64_t x) {
  if ((s * x) >> 32) { fprintf(stderr, "fu operand overflow %llu*%llu\n", (unsigned long long)s, (unsigned long long)x); abort(); }
  return (uint32_t)(s * x);
}
inline uint64_t at2v_umad_checked(uint64_t a, uint64_t b, uint64_t c) {
  const unsigned __int128 r = (unsigned __int128)a * b + c;
  if ((uint64_t)(r >> 64)) { fprintf(stderr, "fu column overflow\n"); abort(); }
  return (uint64_t)r;
}
inline uint32_t at2v_unarrow_checked(uint64_t c) {
  if (c >> 32) { fprintf(stderr, "fu narrow wrap overflow %llu\n", (unsigned long long)c); abort(); }
  return (uint32_t)c;
}
#define AT2V_UMAD(a, b, c) at2v_umad_checked((uint32_t)(a), (uint32_t)(b), (uint64_t)(c))
#define AT2V_USC(s, x) at2v_usc_checked((s), (x))
#define AT2V_UNARROW(c) at2v_unarrow_checked(c)
#else
#define AT2V_UMAD(a, b, c) ((uint64_t)(uint32_t)(a) * (uint64_t)(uint32_t)(b) + (uint64_t)(c))
#define AT2V_USC(s, x) ((s) * (x))
// top carry known (tools/gen_fu.py check_group_law) to be below 2^32: the one-MAD wrap
#define AT2V_UNARROW(c) ((uint32_t)(c))
#endif

#if defined(__HIP_DEVICE_COMPILE__)
// 2*x as a full-rate v_add_u32 (LLVM would emit the half-rate v_lshlrev_b32 on gfx950)
__device__ AT2V_INLINE uint32_t at2v_udbl32(uint32_t x) {
  uint32_t r;
  asm("v_add_u32 %0, %1, %1" : "=v"(r) : "v"(x));
  return r;
}
#define AT2V_UX2(x) at2v_udbl32(x)
#ifndef AT2V_FU_ASM
#define AT2V_FU_ASM 1
#endif
// AT2V_FU_FUSED = 1: every single product is ONE asm statement (accumulator in the clobbered pair v[254:255], limbs and
// carries extracted inside the string), so hipcc's one-state pad after each inline asm (an s_nop 0 before the carry
// shift) comes once per product instead of once per column (tools/gen_fu.py emit_fused)
#ifndef AT2V_FU_FUSED
#define AT2V_FU_FUSED 0
#endif
#else
#define AT2V_UX2(x) AT2V_USC(2u, (x))
#undef AT2V_FU_ASM
#define AT2V_FU_ASM 0
#endif

#define AT2V_FU_CONST constexpr

namespace at2v {

struct fu {
  uint32_t v[10];
};

}  // namespace at2v
