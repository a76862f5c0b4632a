// Phase breakdown of the verify kernel on gfx950: the product kernel (at2v_kernels.hip, included
// verbatim) built with AT2V_PHASE(k) = "lane 0 adds the s_memtime delta since the previous mark to
// bucket k of its wave". Buckets (full-length path): 0 loop/pair overhead, 1 loads + V1 + decompress A,
// 2 SHA-512 + mod l + recode, 3 A table, 4 ladder, 5 group inversion, 6 encode + compare + verdict store;
// (half-size path): 1 adds decoding R, 2 adds the lattice reduction, 3 builds both tables, 6 = identity check.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I at2-node_amd/csrc tools/phase_bench.hip -o tools/phase_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <vector>

#define AT2V_MAX_WAVES 4096
__device__ unsigned long long at2v_phase_acc[AT2V_MAX_WAVES][8];
__device__ unsigned long long at2v_phase_last[AT2V_MAX_WAVES];
// first and last mark of every wave on the constant-rate, device-wide wall clock (s_memrealtime, 100 MHz):
// the spread of wave end times is the kernel's tail (waves idle while the slowest finish)
__device__ unsigned long long at2v_wave_t0[AT2V_MAX_WAVES];
__device__ unsigned long long at2v_wave_t1[AT2V_MAX_WAVES];
__device__ __forceinline__ void at2v_phase_mark(int k) {
  const unsigned w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if ((threadIdx.x & 63) == 0 && w < AT2V_MAX_WAVES) {
    const unsigned long long wt = wall_clock64();
    if (at2v_wave_t0[w] == 0) at2v_wave_t0[w] = wt;
    at2v_wave_t1[w] = wt;
    const unsigned long long t = clock64();
    if (k > 0) at2v_phase_acc[w][k] += t - at2v_phase_last[w];
    else if (at2v_phase_last[w]) at2v_phase_acc[w][0] += t - at2v_phase_last[w];
    at2v_phase_last[w] = t;
  }
}
#ifdef AT2V_WAIT_PROBE
// s_waitcnt probe build (no phase marks, so no extra memory operations in the measured waves): per-chunk sums of the
// cycles spent in the A/R entry waits, the B entry waits, the digit-word reads and the mid-window pacing mark, and
// the chunk's total, summed over all chunks
__device__ unsigned long long at2v_probe_acc[7];
#define AT2V_WAIT_PROBE_SINK(a, b, c, d, e, f, g) \
  do {                                           \
    if ((threadIdx.x & 63) == 0) {               \
      atomicAdd(&at2v_probe_acc[0], (a));        \
      atomicAdd(&at2v_probe_acc[1], (b));        \
      atomicAdd(&at2v_probe_acc[2], (c));        \
      atomicAdd(&at2v_probe_acc[3], (d));        \
      atomicAdd(&at2v_probe_acc[4], (e));        \
      atomicAdd(&at2v_probe_acc[5], (f));        \
      atomicAdd(&at2v_probe_acc[6], (g));        \
    }                                            \
  } while (0)
#else
#define AT2V_PHASE(k) at2v_phase_mark(k)
#endif

#include "at2v_kernels.hip"

#define CHECK(x)                                                               \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      printf("HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                                \
    }                                                                          \
  } while (0)

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : (1u << 20);
  // launches of <= pair_max records run the two-lanes-per-record kernel (0: always the throughput kernel)
  const uint32_t pair_max = argc > 2 ? (uint32_t)atoi(argv[2]) : 0u;
  const uint32_t L = 100;
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  int bpc = 0, vg = 0;
  CHECK(at2v::verify_occupancy(&bpc, &vg));
  const int grid = prop.multiProcessorCount * bpc;
  const int wpb = at2v::block_threads() / 64;
  if (grid * wpb > AT2V_MAX_WAVES) {
    printf("grid too large\n");
    return 1;
  }
  uint8_t *pk, *sig, *msg;
  uint32_t *off, *ver;
  int4 *scratch, *btab;
  CHECK(hipMalloc(&pk, (size_t)n * 32));
  CHECK(hipMalloc(&sig, (size_t)n * 64));
  CHECK(hipMalloc(&msg, (size_t)n * L));
  CHECK(hipMalloc(&off, (size_t)(n + 1) * 4));
  CHECK(hipMalloc(&ver, (size_t)(n + 31) / 32 * 4));
  CHECK(hipMalloc(&scratch, at2v::scratch_bytes(grid)));
  CHECK(hipMalloc(&btab, at2v::btab_bytes()));
  CHECK(at2v::launch_build_btab(btab, 0));
  CHECK(at2v::launch_gen(0x4154325F, 0, n, L, pk, sig, msg, off, 0));
  CHECK(hipDeviceSynchronize());
  std::vector<unsigned long long> zero(AT2V_MAX_WAVES * 8, 0), zl(AT2V_MAX_WAVES, 0);
  float ms = 0;
  for (int rep = 0; rep < 2; ++rep) {
    CHECK(hipMemcpyToSymbol(HIP_SYMBOL(at2v_phase_acc), zero.data(), zero.size() * 8));
#ifdef AT2V_WAIT_PROBE
    CHECK(hipMemcpyToSymbol(HIP_SYMBOL(at2v_probe_acc), zero.data(), 7 * 8));
#endif
    CHECK(hipMemcpyToSymbol(HIP_SYMBOL(at2v_phase_last), zl.data(), zl.size() * 8));
    CHECK(hipMemcpyToSymbol(HIP_SYMBOL(at2v_wave_t0), zl.data(), zl.size() * 8));
    CHECK(hipMemcpyToSymbol(HIP_SYMBOL(at2v_wave_t1), zl.data(), zl.size() * 8));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    CHECK(hipEventRecord(e0, 0));
    CHECK(at2v::launch_verify(pk, sig, msg, n * L, off, n, 0, ver, scratch, btab, grid, pair_max, 0));
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms, e0, e1));
  }
  std::vector<unsigned long long> acc(AT2V_MAX_WAVES * 8);
  CHECK(hipMemcpyFromSymbol(acc.data(), HIP_SYMBOL(at2v_phase_acc), acc.size() * 8));
  std::vector<uint32_t> hv((n + 31) / 32);
  CHECK(hipMemcpy(hv.data(), ver, hv.size() * 4, hipMemcpyDeviceToHost));
  size_t valid = 0;
  for (uint32_t i = 0; i < n; ++i) valid += (hv[i / 32] >> (i % 32)) & 1;
#if AT2V_VERIFY_HALF
  const char* names[8] = {"loop overhead", "loads+V1+decode A,R", "t = c1 s mod l + recode", "A,R tables",
                          "ladder", "sha512 + mod l", "identity check+store", "lattice reduction"};
#else
  const char* names[8] = {"pair/loop overhead", "loads+V1+decompress", "sha512+mod l+recode", "A table",
                          "ladder", "group inversion", "encode+compare+store", "-"};
#endif
  double tot = 0, b[8] = {0};
  const int waves = grid * wpb;
  for (int w = 0; w < waves; ++w)
    for (int k = 0; k < 8; ++k) b[k] += (double)acc[w * 8 + k];
  for (int k = 0; k < 8; ++k) tot += b[k];
  printf("n=%u grid=%d waves=%d kernel %.3f ms -> %.2f M verifies/s, valid %zu/%u\n", n, grid, waves, ms,
         n / ms / 1e3, valid, n);
  const double chunks = (double)n / 64;
  for (int k = 0; k < 8; ++k)
    printf("  %-24s %6.2f %%   %10.0f wave-cycles per 64-record chunk\n", names[k], 100 * b[k] / tot, b[k] / chunks);
  printf("  total                    %10.0f wave-cycles per chunk (s_memtime; 2 waves share a SIMD)\n", tot / chunks);
#ifdef AT2V_WAIT_PROBE
  {
    unsigned long long pa[7];
    CHECK(hipMemcpyFromSymbol(pa, HIP_SYMBOL(at2v_probe_acc), sizeof(pa)));
    const char* pn[7] = {"A/R entry waits", "B entry waits", "digit-word reads (loop top)", "mid-window pacing mark",
                         "-", "A/R entry LDS reads (lgkm)", "chunk-start input loads"};
    for (int k = 0; k < 7; ++k) {
      if (k == 4) continue;
      printf("  probe %-28s %6.2f %% of chunk time  (%10.0f cycles per chunk)\n", pn[k], 100.0 * pa[k] / pa[4],
             pa[k] / chunks);
    }
    printf("  probe chunk total %10.0f cycles per chunk\n", pa[4] / chunks);
  }
#endif
#ifndef AT2V_WAIT_PROBE  // the probe build sets no marks: no per-wave timeline
  {
    std::vector<unsigned long long> t0(AT2V_MAX_WAVES), t1(AT2V_MAX_WAVES);
    CHECK(hipMemcpyFromSymbol(t0.data(), HIP_SYMBOL(at2v_wave_t0), t0.size() * 8));
    CHECK(hipMemcpyFromSymbol(t1.data(), HIP_SYMBOL(at2v_wave_t1), t1.size() * 8));
    unsigned long long s0 = ~0ull, s1 = 0, e0 = ~0ull, e1 = 0;
    std::vector<double> ends;
    double life = 0;
    for (int w = 0; w < waves; ++w) {
      if (!t0[w]) continue;
      s0 = t0[w] < s0 ? t0[w] : s0;
      s1 = t0[w] > s1 ? t0[w] : s1;
      e0 = t1[w] < e0 ? t1[w] : e0;
      e1 = t1[w] > e1 ? t1[w] : e1;
    }
    for (int w = 0; w < waves; ++w)
      if (t0[w]) {
        ends.push_back((double)(t1[w] - s0));
        life += (double)(t1[w] - t0[w]);
      }
    std::sort(ends.begin(), ends.end());
    const double span = (double)(e1 - s0), m = ends.size();
    printf("wave timeline (100 MHz wall clock, us from the first wave's first mark): start spread %.1f us; end min %.1f "
           "p10 %.1f p50 %.1f p90 %.1f p99 %.1f max %.1f; mean wave life / span = %.4f\n",
           (s1 - s0) / 100.0, ends[0] / 100, ends[(size_t)(0.1 * m)] / 100, ends[(size_t)(0.5 * m)] / 100,
           ends[(size_t)(0.9 * m)] / 100, ends[(size_t)(0.99 * m)] / 100, span / 100, life / m / span);
  }
#endif
  return valid == n ? 0 : 2;
}
