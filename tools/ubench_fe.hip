// Field-op microbenchmark on gfx950: cycles per fe_mul / fe_sq in a long dependent chain,
// many waves per SIMD. Build: hipcc --offload-arch=gfx950 -O3 -I at2-node_amd/csrc tools/ubench_fe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include "at2v_fe.h"
using namespace at2v;

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e_)); return 1; } } while (0)

template <int OP, int WPS>
__global__ __launch_bounds__(256, WPS) void kern(int32_t* out, int iters, int32_t seed) {
  fe a, b, c;
  for (int i = 0; i < 10; ++i) { a.v[i] = (seed * (i + 3) + threadIdx.x) & 0xffffff; b.v[i] = (seed ^ (i * 77)) & 0xffffff; c.v[i] = i; }
  for (int it = 0; it < iters; ++it) {
    if constexpr (OP == 0) { fe_mul(a, a, b); }
    if constexpr (OP == 1) { fe_sq(a, a); }
    if constexpr (OP == 2) { fe_mul(a, a, b); fe_mul(c, c, b); }   // two independent chains
    if constexpr (OP == 3) {  // mads only (no carry): 100 mads -> fold to 32 bits by truncation
      int64_t h[10];
#pragma unroll
      for (int k = 0; k < 10; ++k) h[k] = 0;
#pragma unroll
      for (int i = 0; i < 10; ++i)
#pragma unroll
        for (int j = 0; j < 10; ++j) h[(i + j) % 10] = AT2V_MAD(a.v[i], b.v[j], h[(i + j) % 10]);
#pragma unroll
      for (int k = 0; k < 10; ++k) a.v[k] = (int32_t)(h[k] >> 20);
    }
    if constexpr (OP == 4) { fe_sq(a, a); fe_sq(c, c); }
  }
  int32_t s = 0;
  for (int i = 0; i < 10; ++i) s += a.v[i] + c.v[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int OP, int WPS>
int run(const char* name, int32_t* d, int cus, int ops_per_iter) {
  const int blocks = cus * WPS;  // 256-thread blocks: WPS waves per SIMD
  const int iters = 2000;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL((kern<OP, WPS>), dim3(blocks), dim3(256), 0, 0, d, 10, 1);
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 3; ++r) {
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL((kern<OP, WPS>), dim3(blocks), dim3(256), 0, 0, d, iters, r + 2);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  // per SIMD: WPS waves x iters x ops field ops, in best ms at ~2.4 GHz nominal clock
  const double ops_per_simd = (double)WPS * iters * ops_per_iter;
  const double cyc = best * 1e-3 * 2.4e9 / ops_per_simd;
  const double rate = (double)blocks * 256 * iters * ops_per_iter / (best * 1e-3);
  printf("%-34s waves/SIMD=%d  %8.3f ms  %7.1f cycles(2.4GHz)/op/SIMD  %.2f Gop/s (lane field ops)\n", name, WPS, best, cyc, rate / 1e9);
  return 0;
}

int main() {
  hipDeviceProp_t p; CHECK(hipGetDeviceProperties(&p, 0));
  int32_t* d; CHECK(hipMalloc(&d, (size_t)p.multiProcessorCount * 8 * 256 * 4));
  const int cus = p.multiProcessorCount;
  run<0, 1>("fe_mul chain", d, cus, 1);
  run<0, 2>("fe_mul chain", d, cus, 1);
  run<0, 4>("fe_mul chain", d, cus, 1);
  run<2, 1>("fe_mul x2 independent", d, cus, 2);
  run<2, 2>("fe_mul x2 independent", d, cus, 2);
  run<1, 1>("fe_sq chain", d, cus, 1);
  run<1, 2>("fe_sq chain", d, cus, 1);
  run<4, 2>("fe_sq x2 independent", d, cus, 2);
  run<3, 1>("100 mads only", d, cus, 1);
  run<3, 2>("100 mads only", d, cus, 1);
  run<3, 4>("100 mads only", d, cus, 1);
  return 0;
}
