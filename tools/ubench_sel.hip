// Select / bit-logic instruction rates on gfx950 (what a conditional negation or a SHA-512 round can be built on).
// Each lane runs CH independent chains of one instruction for ITERS iterations at 2 waves/SIMD (8 waves/CU);
// result = lane-instructions per second over the whole chip, and the fraction of the full-rate peak
// (256 CU x 128 lanes/clk x 2.4 GHz).  Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_sel.hip -o tools/ubench_sel
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP %s @%d: %s\n", #x, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

constexpr int ITERS = 8192;
constexpr int CH = 8;

#define BODY(ASM, ...) \
  _Pragma("unroll") for (int c = 0; c < CH; ++c) { asm volatile(ASM : "+v"(r[c]) : __VA_ARGS__); }

template <int OP>
__global__ __launch_bounds__(256) void kern(uint32_t* out, uint32_t a0, uint32_t b0) {
  uint32_t r[CH];
  uint32_t a = a0 ^ threadIdx.x, b = b0 + threadIdx.x;
  const uint32_t m = (threadIdx.x & 1) ? 0xffffffffu : 0u;  // per-lane all-ones / all-zeros mask
  uint64_t sm;  // lane mask in an SGPR pair
  asm volatile("v_cmp_ne_u32 %0, 0, %1" : "=s"(sm) : "v"(m));
#pragma unroll
  for (int c = 0; c < CH; ++c) r[c] = a + c;
  for (int it = 0; it < ITERS; ++it) {
    if constexpr (OP == 0) { BODY("v_add_u32 %0, %1, %0", "v"(a)) }
    if constexpr (OP == 1) { BODY("v_cndmask_b32_e64 %0, %1, %0, %2", "v"(a), "s"(sm)) }
    if constexpr (OP == 2) {
#pragma unroll
      for (int c = 0; c < CH; ++c) asm volatile("s_mov_b64 vcc, %2\n\tv_cndmask_b32 %0, %1, %0, vcc" : "+v"(r[c]) : "v"(a), "s"(sm) : "vcc");
    }
    if constexpr (OP == 3) { BODY("v_bfi_b32 %0, %1, %2, %0", "v"(m), "v"(a)) }
    if constexpr (OP == 4) { BODY("v_bitop3_b32 %0, %1, %2, %0 bitop3:0x96", "v"(a), "v"(b)) }
    if constexpr (OP == 5) { BODY("v_perm_b32 %0, %1, %0, %2", "v"(a), "v"(b)) }
    if constexpr (OP == 6) { BODY("v_lshrrev_b32 %0, 3, %0", "v"(a)) }
    if constexpr (OP == 7) { BODY("v_or_b32 %0, %1, %0", "v"(a)) }
    if constexpr (OP == 8) { BODY("v_and_or_b32 %0, %1, %2, %0", "v"(a), "v"(b)) }
    if constexpr (OP == 9) { BODY("v_or3_b32 %0, %1, %2, %0", "v"(a), "v"(b)) }
    if constexpr (OP == 10) { BODY("v_xad_u32 %0, %1, %2, %0", "v"(a), "v"(b)) }
    if constexpr (OP == 11) { BODY("v_mov_b32 %0, %1", "v"(r[(c + 1) % CH])) }
    if constexpr (OP == 12) { BODY("v_max_u32 %0, %1, %0", "v"(a)) }
    if constexpr (OP == 13) { BODY("v_sub_u32 %0, %1, %0", "v"(a)) }
    if constexpr (OP == 14) { BODY("v_cndmask_b32_e64 %0, %1, %0, %2", "v"(a), "s"(sm)) }  // same as 1, repeated
    if constexpr (OP == 15) { BODY("v_bitop3_b32 %0, %1, %2, %0 bitop3:0xe8", "v"(a), "v"(b)) }
  }
  uint32_t acc = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) acc += r[c];
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

static const char* NAMES[] = {"v_add_u32", "v_cndmask_b32_e64 (sgpr mask)", "s_mov vcc + v_cndmask_b32 (vcc)",
                              "v_bfi_b32 (vgpr mask)", "v_bitop3_b32 0x96 (xor3)", "v_perm_b32", "v_lshrrev_b32",
                              "v_or_b32", "v_and_or_b32", "v_or3_b32", "v_xad_u32", "v_mov_b32", "v_max_u32",
                              "v_sub_u32", "v_cndmask_b32_e64 (again)", "v_bitop3_b32 0xe8 (maj)"};

template <int OP>
int run(uint32_t* dout, int blocks) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(256), 0, 0, dout, 12345u, 6789u);
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(256), 0, 0, dout, 12345u + rep, 6789u);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  const double n = (double)blocks * 256 * ITERS * CH;
  const double rate = n / (best * 1e-3);
  printf("%-34s %8.3f ms  %8.2f Tlane-op/s  (%.3f of 7.86e13 full-rate)\n", NAMES[OP], best, rate / 1e12,
         rate / 7.864e13);
  return 0;
}

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  printf("device %s CUs=%d\n", p.gcnArchName, p.multiProcessorCount);
  const int blocks = p.multiProcessorCount * 8;  // 256-thread blocks, 8 per CU = 2 waves per SIMD
  uint32_t* dout;
  CHECK(hipMalloc(&dout, (size_t)blocks * 256 * 4));
  run<0>(dout, blocks); run<1>(dout, blocks); run<2>(dout, blocks); run<3>(dout, blocks);
  run<4>(dout, blocks); run<5>(dout, blocks); run<6>(dout, blocks); run<7>(dout, blocks);
  run<8>(dout, blocks); run<9>(dout, blocks); run<10>(dout, blocks); run<11>(dout, blocks);
  run<12>(dout, blocks); run<13>(dout, blocks); run<14>(dout, blocks); run<15>(dout, blocks);
  CHECK(hipFree(dout));
  return 0;
}
