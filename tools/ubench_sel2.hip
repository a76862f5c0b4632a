// v_cndmask_b32 cost in a realistic mix on gfx950: VOP2 form (mask in VCC, written by a v_cmp) against the VOP3 form
// (mask in an SGPR pair), alone and interleaved with independent v_mad_u64_u32 chains, 2 waves/SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_sel2.hip -o tools/ubench_sel2
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP %s @%d: %s\n", #x, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

constexpr int ITERS = 4096;

template <int OP>
__global__ __launch_bounds__(256) void kern(uint32_t* out, uint32_t a0, uint32_t b0) {
  uint32_t r[8];
  uint64_t q[16];
  uint32_t a = a0 ^ threadIdx.x, b = b0 + threadIdx.x;
  const int d = (int)(threadIdx.x & 15) - 7;
#pragma unroll
  for (int c = 0; c < 8; ++c) r[c] = a + c;
#pragma unroll
  for (int c = 0; c < 16; ++c) q[c] = (uint64_t)b * (c + 1);
  for (int it = 0; it < ITERS; ++it) {
    if constexpr (OP == 0 || OP == 2) {  // 16 independent MADs
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        uint64_t cy;
        asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(q[c]), "=s"(cy) : "v"(a), "v"(b));
      }
    }
    if constexpr (OP == 0 || OP == 1) {  // v_cmp -> vcc, 8 VOP2 selects on vcc
      asm volatile("v_cmp_gt_i32 vcc, 0, %0" : : "v"(d + it) : "vcc");
#pragma unroll
      for (int c = 0; c < 8; ++c) asm volatile("v_cndmask_b32 %0, %1, %0, vcc" : "+v"(r[c]) : "v"(a) : "vcc");
    }
    if constexpr (OP == 2 || OP == 3) {  // v_cmp -> sgpr pair, 8 VOP3 selects on it
      uint64_t m;
      asm volatile("v_cmp_gt_i32_e64 %0, 0, %1" : "=s"(m) : "v"(d + it));
#pragma unroll
      for (int c = 0; c < 8; ++c) asm volatile("v_cndmask_b32_e64 %0, %1, %0, %2" : "+v"(r[c]) : "v"(a), "s"(m));
    }
    if constexpr (OP == 4) {  // MADs only
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        uint64_t cy;
        asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(q[c]), "=s"(cy) : "v"(a), "v"(b));
      }
    }
    if constexpr (OP == 5) {  // v_cmp -> vcc and 8 selects written as C (what LLVM emits for `neg ? b : a`)
      const bool neg = (d + it) < 0;
#pragma unroll
      for (int c = 0; c < 8; ++c) { r[c] = neg ? a : r[c]; asm volatile("" : "+v"(r[c])); }
    }
  }
  uint32_t acc = 0;
#pragma unroll
  for (int c = 0; c < 8; ++c) acc += r[c];
#pragma unroll
  for (int c = 0; c < 16; ++c) acc += (uint32_t)q[c];
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

static const char* NAMES[] = {"16 MAD + cmp + 8 cndmask(vcc)", "cmp + 8 cndmask(vcc)", "16 MAD + cmp + 8 cndmask_e64(sgpr)",
                              "cmp + 8 cndmask_e64(sgpr)", "16 MAD", "cmp + 8 selects (compiler)"};

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
  // SIMD-cycles per iteration per wave pair, at an assumed 2.1 GHz: time * clk / (iterations * waves per SIMD pair)
  const double waves_per_simd = (double)blocks * 4 / (256 * 4);
  printf("%-40s %8.3f ms   %7.1f ns per iteration per SIMD\n", NAMES[OP], best,
         best * 1e6 / (ITERS * waves_per_simd));
  return 0;
}

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  printf("device %s CUs=%d\n", p.gcnArchName, p.multiProcessorCount);
  const int blocks = p.multiProcessorCount * 8;
  uint32_t* dout;
  CHECK(hipMalloc(&dout, (size_t)blocks * 256 * 4));
  run<4>(dout, blocks); run<0>(dout, blocks); run<2>(dout, blocks); run<1>(dout, blocks); run<3>(dout, blocks);
  run<5>(dout, blocks);
  CHECK(hipFree(dout));
  return 0;
}
