// Field-op microbenchmark on gfx950: the balanced signed field (at2v_fe_gen.h: column-interleaved MADs, separate
// carry chain) against the unsigned chained-carry field (at2v_fu_gen.h: each column's MAD chain starts from the
// previous column's carry). Cycles per op in long dependent chains at 1 and 2 waves per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I at2-node_amd/csrc tools/ubench_fu.hip -o tools/ubench_fu
#include <hip/hip_runtime.h>
#include <cstdio>
#include "at2v_fe.h"
#include "at2v_ge.h"
#include "at2v_fu_gen.h"
using namespace at2v;

// doubling prototype on the unsigned field (p2 -> p1p1 -> p2); K1, K2 are multiples of p with large limbs
__device__ __forceinline__ void fu_dbl_p2(fu& X, fu& Y, fu& Z) {
  constexpr uint32_t K1[10] = {0x7ffffdau, 0x3fffffeu, 0x7fffffeu, 0x3fffffeu, 0x7fffffeu, 0x3fffffeu, 0x7fffffeu, 0x3fffffeu, 0x7fffffeu, 0x3fffffeu};
  constexpr uint32_t K2[10] = {0xbffffc7u, 0x5fffffdu, 0xbfffffdu, 0x5fffffdu, 0xbfffffdu, 0x5fffffdu, 0xbfffffdu, 0x5fffffdu, 0xbfffffdu, 0x5fffffdu};
  fu s, XX, YY, t0, ZZ2, E, G, F, H;
#pragma unroll
  for (int i = 0; i < 10; ++i) s.v[i] = X.v[i] + Y.v[i];
  fu_sq_x2(XX, X, YY, Y);
  fu_sq_sq2(t0, s, ZZ2, Z);
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    H.v[i] = XX.v[i] + YY.v[i];
    E.v[i] = t0.v[i] + K2[i] - H.v[i];
    G.v[i] = YY.v[i] + K1[i] - XX.v[i];
    F.v[i] = ZZ2.v[i] + K2[i] - G.v[i];
  }
  fu_mul_x2(X, E, F, Y, G, H);
  fu_mul(Z, F, G);
}

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e_)); return 1; } } while (0)

template <int OP, int WPS>
__global__ __launch_bounds__(256, WPS) void kern(uint32_t* out, int iters, int32_t seed) {
  fe a, b, c;
  fu x, y, z;
  for (int i = 0; i < 10; ++i) {
    a.v[i] = (seed * (i + 3) + threadIdx.x) & 0xffffff; b.v[i] = (seed ^ (i * 77)) & 0xffffff; c.v[i] = i;
    x.v[i] = (uint32_t)a.v[i]; y.v[i] = (uint32_t)b.v[i]; z.v[i] = i;
  }
  for (int it = 0; it < iters; ++it) {
    if constexpr (OP == 0) { fe_mul(a, a, b); }
    if constexpr (OP == 1) { fe_sq(a, a); }
    if constexpr (OP == 2) { fe_sq(a, a); fe_sq(c, c); fe_mul(b, a, c); }
    if constexpr (OP == 10) { fu_mul(x, x, y); }
    if constexpr (OP == 11) { fu_sq(x, x); }
    if constexpr (OP == 12) { fu_sq(x, x); fu_sq(z, z); fu_mul(y, x, z); }
    if constexpr (OP == 3) { fe_sq(a, a); fe_sq(c, c); }
    if constexpr (OP == 4) { fe_mul(a, a, b); fe_mul(c, c, b); }
    if constexpr (OP == 13) { fu_sq_x2(x, x, z, z); }
    if constexpr (OP == 14) { fu_mul_x2(x, x, y, z, z, y); }
    if constexpr (OP == 20) { ge_p2 q{a, b, c}; ge_p1p1 t; ge_p2_dbl(t, q); ge_p1p1_to_p2(q, t); a = q.X; b = q.Y; c = q.Z; }
    if constexpr (OP == 21) { fu_dbl_p2(x, y, z); }
  }
  uint32_t s = 0;
  for (int i = 0; i < 10; ++i) s += (uint32_t)a.v[i] + (uint32_t)b.v[i] + (uint32_t)c.v[i] + x.v[i] + y.v[i] + z.v[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int OP, int WPS>
int run(const char* name, uint32_t* d, int cus, int ops_per_iter) {
  const int blocks = cus * WPS;  // 256-thread blocks: WPS waves per SIMD
  const int iters = 4000;
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
  const double ops_per_simd = (double)WPS * iters * ops_per_iter;
  const double cyc = best * 1e-3 * 2.4e9 / ops_per_simd;
  printf("%-40s waves/SIMD=%d  %8.3f ms  %7.1f cycles(2.4GHz)/op/SIMD\n", name, WPS, best, cyc);
  return 0;
}

int main() {
  hipDeviceProp_t p; CHECK(hipGetDeviceProperties(&p, 0));
  uint32_t* d; CHECK(hipMalloc(&d, (size_t)p.multiProcessorCount * 8 * 256 * 4));
  const int cus = p.multiProcessorCount;
  run<0, 2>("fe_mul chain (signed, balanced)", d, cus, 1);
  run<10, 2>("fu_mul chain (unsigned, chained carry)", d, cus, 1);
  run<1, 2>("fe_sq chain (signed, balanced)", d, cus, 1);
  run<11, 2>("fu_sq chain (unsigned, chained carry)", d, cus, 1);
  run<2, 2>("fe 2 sq + 1 mul", d, cus, 3);
  run<12, 2>("fu 2 sq + 1 mul", d, cus, 3);
  run<3, 2>("fe_sq x2 independent", d, cus, 2);
  run<13, 2>("fu_sq_x2 (interleaved pair)", d, cus, 2);
  run<4, 2>("fe_mul x2 independent", d, cus, 2);
  run<14, 2>("fu_mul_x2 (interleaved pair)", d, cus, 2);
  run<20, 2>("fe doubling p2->p2 (4S+3M)", d, cus, 1);
  run<21, 2>("fu doubling p2->p2 (4S+3M)", d, cus, 1);
  run<0, 1>("fe_mul chain (signed, balanced)", d, cus, 1);
  run<10, 1>("fu_mul chain (unsigned, chained carry)", d, cus, 1);
  run<1, 1>("fe_sq chain (signed, balanced)", d, cus, 1);
  run<11, 1>("fu_sq chain (unsigned, chained carry)", d, cus, 1);
  return 0;
}
