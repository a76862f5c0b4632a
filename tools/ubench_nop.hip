// Cost of the s_nop LLVM places after an inline-asm block whose output the next instruction reads (gfx950, 2 waves
// per SIMD): the same column-chain work (10 columns x 10 dependent v_mad_u64_u32 + a 64-bit shift per column) as
// one asm block per column (LLVM inserts an s_nop before each shift) against one asm block for all columns.
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_nop.hip -o tools/ubench_nop
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP %s @%d: %s\n", #x, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

constexpr int ITERS = 2048;

#define MAD10(D, A, B, C)                                                                                         \
  "v_mad_u64_u32 " D ", vcc, " A ", " B ", " C "\n\tv_mad_u64_u32 " D ", vcc, " B ", " A ", " D "\n\t"             \
  "v_mad_u64_u32 " D ", vcc, " A ", " B ", " D "\n\tv_mad_u64_u32 " D ", vcc, " B ", " A ", " D "\n\t"               \
  "v_mad_u64_u32 " D ", vcc, " A ", " B ", " D "\n\tv_mad_u64_u32 " D ", vcc, " B ", " A ", " D "\n\t"               \
  "v_mad_u64_u32 " D ", vcc, " A ", " B ", " D "\n\tv_mad_u64_u32 " D ", vcc, " B ", " A ", " D "\n\t"               \
  "v_mad_u64_u32 " D ", vcc, " A ", " B ", " D "\n\tv_mad_u64_u32 " D ", vcc, " B ", " A ", " D "\n\t"

template <int OP>
__global__ __launch_bounds__(512) void kern(uint64_t* out, uint32_t a0, uint32_t b0) {
  uint32_t a = a0 ^ threadIdx.x, b = b0 + threadIdx.x;
  uint64_t c0 = a, c1 = b;
  for (int it = 0; it < ITERS; ++it) {
    if constexpr (OP == 0) {  // one asm per column: the shift after each block reads its output
#pragma unroll
      for (int k = 0; k < 10; ++k) {
        uint64_t h0, h1;
        asm(MAD10("%0", "%2", "%3", "%4") MAD10("%1", "%3", "%2", "%5") : "=&v"(h0), "=&v"(h1)
            : "v"(a), "v"(b), "v"(c0), "v"(c1) : "vcc");
        c0 = h0 >> 26;
        c1 = h1 >> 25;
      }
    }
    if constexpr (OP == 1) {  // the same instructions, shifts included, as one asm block
      uint64_t h0, h1;
#define COL MAD10("%0", "%4", "%5", "%2") MAD10("%1", "%5", "%4", "%3") \
            "v_lshrrev_b64 %2, 26, %0\n\tv_lshrrev_b64 %3, 25, %1\n\t"
      asm(COL COL COL COL COL COL COL COL COL COL : "=&v"(h0), "=&v"(h1), "+v"(c0), "+v"(c1) : "v"(a), "v"(b) : "vcc");
#undef COL
    }
  }
  out[blockIdx.x * 512 + threadIdx.x] = c0 + c1;
}

template <int OP>
int run(uint64_t* dout, int blocks, const char* name) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(512), 0, 0, dout, 12345u, 6789u);
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(kern<OP>, dim3(blocks), dim3(512), 0, 0, dout, 12345u + rep, 6789u);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  const double inst = (double)blocks * 8 * ITERS * 10 * 22;  // wave-instructions (MADs + shifts)
  printf("%-44s %8.3f ms   %.2f ns per 1k wave-instructions per SIMD\n", name, best, best * 1e6 / (inst / 1024) * 1e3);
  return 0;
}

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  printf("device %s CUs=%d, 512-thread blocks, one per CU (2 waves per SIMD)\n", p.gcnArchName, p.multiProcessorCount);
  const int blocks = p.multiProcessorCount;
  uint64_t* dout;
  CHECK(hipMalloc(&dout, (size_t)blocks * 512 * 8));
  run<0>(dout, blocks, "asm per column (s_nop before each shift)");
  run<1>(dout, blocks, "one asm block (no s_nop)");
  run<0>(dout, blocks, "asm per column (again)");
  run<1>(dout, blocks, "one asm block (again)");
  CHECK(hipFree(dout));
  return 0;
}
