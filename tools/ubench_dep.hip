// Dependency-latency microbenchmark on gfx950: issue rate of v_mad_i64_i32 and of the carry step
// (v_ashrrev_i64 + v_lshl_add_u64) with K independent chains per lane at W waves per SIMD, and
// v_cndmask_b32 with an SGPR-pair mask. Build: hipcc -O3 --offload-arch=gfx950 tools/ubench_dep.hip -o tools/ubench_dep
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CHECK(x)                                                        \
  do {                                                                  \
    hipError_t e_ = (x);                                                \
    if (e_ != hipSuccess) {                                             \
      fprintf(stderr, "HIP %s @%d: %s\n", #x, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                         \
    }                                                                   \
  } while (0)

constexpr int ITERS = 4096;

template <int OP, int K>
__global__ __launch_bounds__(256) void kern(uint32_t* out, uint32_t a0, uint32_t b0) {
  uint64_t q[K];
  uint32_t r[K];
  const uint32_t a = a0 ^ threadIdx.x, b = b0 + threadIdx.x;
  const uint64_t m = (blockIdx.x & 1) ? 0x5555555555555555ull : 0xaaaaaaaaaaaaaaaaull;
#pragma unroll
  for (int c = 0; c < K; ++c) {
    q[c] = (uint64_t)b * (c + 1);
    r[c] = a + c;
  }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int rep = 0; rep < 12 / K + 1; ++rep) {
#pragma unroll
      for (int c = 0; c < K; ++c) {
        if constexpr (OP == 0) {
          uint64_t cy;
          asm volatile("v_mad_i64_i32 %0, %1, %2, %3, %0" : "+v"(q[c]), "=s"(cy) : "v"(a), "v"(b));
        }
        if constexpr (OP == 1) {  // carry step: c = q >> 26; q' = c + q
          asm volatile("v_ashrrev_i64 v[254:255], 26, %0\n\tv_lshl_add_u64 %0, v[254:255], 0, %0"
                       : "+v"(q[c])
                       :
                       : "v254", "v255");
        }
        if constexpr (OP == 2) asm volatile("v_cndmask_b32_e64 %0, %1, %0, %2" : "+v"(r[c]) : "v"(a), "s"(m));
        if constexpr (OP == 3) asm volatile("v_add_u32 %0, %1, %0" : "+v"(r[c]) : "v"(a));
      }
    }
  }
  uint32_t acc = 0;
#pragma unroll
  for (int c = 0; c < K; ++c) acc += (uint32_t)q[c] + (uint32_t)(q[c] >> 32) + r[c];
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int OP, int K>
int run(const char* name, uint32_t* dout, int cus, int wps) {
  const int blocks = cus * wps;  // 256-thread blocks: wps waves per SIMD
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL((kern<OP, K>), dim3(blocks), dim3(256), 0, 0, dout, 1u, 2u);
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 3; ++rep) {
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL((kern<OP, K>), dim3(blocks), dim3(256), 0, 0, dout, 3u + rep, 5u);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  const double insts_per_wave = (double)ITERS * (12 / K + 1) * K * (OP == 1 ? 2 : 1);
  const double cyc = best * 1e-3 * 2.4e9 / (insts_per_wave * wps);  // SIMD cycles per wave-instruction
  printf("%-34s K=%2d waves/SIMD=%d  %7.3f ms  %5.2f cycles/instr/SIMD\n", name, K, wps, best, cyc);
  return 0;
}

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  uint32_t* dout;
  CHECK(hipMalloc(&dout, (size_t)cus * 8 * 256 * 4));
  for (int w : {1, 2, 3}) {
    run<0, 1>("v_mad_i64_i32", dout, cus, w);
    run<0, 2>("v_mad_i64_i32", dout, cus, w);
    run<0, 3>("v_mad_i64_i32", dout, cus, w);
    run<0, 4>("v_mad_i64_i32", dout, cus, w);
    run<0, 6>("v_mad_i64_i32", dout, cus, w);
    run<0, 10>("v_mad_i64_i32", dout, cus, w);
    run<1, 1>("carry step (ashr64 + lshl_add_u64)", dout, cus, w);
    run<1, 2>("carry step (ashr64 + lshl_add_u64)", dout, cus, w);
    run<1, 4>("carry step (ashr64 + lshl_add_u64)", dout, cus, w);
    run<1, 8>("carry step (ashr64 + lshl_add_u64)", dout, cus, w);
    run<2, 1>("v_cndmask_b32_e64 sgpr mask", dout, cus, w);
    run<2, 4>("v_cndmask_b32_e64 sgpr mask", dout, cus, w);
    run<3, 1>("v_add_u32", dout, cus, w);
    run<3, 4>("v_add_u32", dout, cus, w);
  }
  CHECK(hipFree(dout));
  return 0;
}
