// Instruction-throughput microbenchmark for gfx950 integer VALU ops that a
// GF(2^255-19) limb design can be built on.
// Each lane runs CH independent dependency chains of one instruction for ITERS
// iterations; result = lane-instructions per second over the whole chip.
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_valu.hip -o tools/ubench_valu
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP %s @%d: %s\n", #x, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

constexpr int ITERS = 16384;
constexpr int CH = 8;

#define BODY32(ASM) \
  _Pragma("unroll") for (int c = 0; c < CH; ++c) { asm volatile(ASM : "+v"(r[c]) : "v"(a), "v"(b)); }

template <int OP>
__global__ __launch_bounds__(256) void kern(uint32_t* out, uint32_t a0, uint32_t b0) {
  uint32_t r[CH];
  uint64_t q[CH];
  double d[CH];
  uint32_t a = a0 ^ threadIdx.x, b = b0 + threadIdx.x;
  double da = (double)a, db = (double)b;
#pragma unroll
  for (int c = 0; c < CH; ++c) { r[c] = a + c; q[c] = (uint64_t)b * (c + 1); d[c] = (double)(c + 1); }
  for (int it = 0; it < ITERS; ++it) {
    if constexpr (OP == 0) { BODY32("v_add_u32 %0, %1, %0") }
    if constexpr (OP == 1) { BODY32("v_mul_lo_u32 %0, %1, %0") }
    if constexpr (OP == 2) { BODY32("v_mul_hi_u32 %0, %1, %0") }
    if constexpr (OP == 3) { BODY32("v_mul_u32_u24 %0, %1, %0") }
    if constexpr (OP == 4) { BODY32("v_mul_hi_u32_u24 %0, %1, %0") }
    if constexpr (OP == 5) { BODY32("v_mad_u32_u24 %0, %1, %2, %0") }
    if constexpr (OP == 6) {
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        uint64_t cy;
        asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(q[c]), "=s"(cy) : "v"(a), "v"(b));
      }
    }
    if constexpr (OP == 7) {
#pragma unroll
      for (int c = 0; c < CH; ++c) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(d[c]) : "v"(da), "v"(db));
    }
    if constexpr (OP == 8) { BODY32("v_dot2_u32_u16 %0, %1, %2, %0") }
    if constexpr (OP == 9) {
#pragma unroll
      for (int c = 0; c < CH; ++c) asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(q[c]) : "v"((uint64_t)a));
    }
    if constexpr (OP == 10) { BODY32("v_add3_u32 %0, %1, %2, %0") }
    if constexpr (OP == 11) { BODY32("v_alignbit_b32 %0, %1, %0, 7") }
    if constexpr (OP == 12) {
#pragma unroll
      for (int c = 0; c < CH; ++c) asm volatile("v_add_co_u32 %0, vcc, %0, %1\n\tv_addc_co_u32 %0, vcc, %0, %2, vcc" : "+v"(r[c]) : "v"(a), "v"(b) : "vcc");
    }
    if constexpr (OP == 13) {
#pragma unroll
      for (int c = 0; c < CH; ++c) asm volatile("v_lshrrev_b64 %0, 7, %0" : "+v"(q[c]));
    }
    if constexpr (OP == 14) { BODY32("v_bfe_u32 %0, %0, 3, 26") }
    if constexpr (OP == 15) {
#pragma unroll
      for (int c = 0; c < CH; ++c) { q[c] = (uint64_t)a * b + q[c]; asm volatile("" : "+v"(q[c])); }
    }
    if constexpr (OP == 16) { BODY32("v_mad_u32_u16 %0, %1, %2, %0") }
    if constexpr (OP == 17) { BODY32("v_lshl_add_u32 %0, %1, 3, %0") }
    if constexpr (OP == 18) { BODY32("v_xor_b32 %0, %1, %0") }
    if constexpr (OP == 19) { BODY32("v_add_u32_e64 %0, %1, %0") }
    if constexpr (OP == 20) {
#pragma unroll
      for (int c = 0; c < CH; ++c) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(r[c]) : "v"(a), "v"(b));
    }
    if constexpr (OP == 21) {
#pragma unroll
      for (int c = 0; c < CH; ++c) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(q[c]) : "v"((uint64_t)a), "v"((uint64_t)b));
    }
    if constexpr (OP == 22) {
#pragma unroll
      for (int c = 0; c < CH; ++c) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(r[c]) : "v"(a) : "vcc");
    }
    if constexpr (OP == 23) { BODY32("v_lshlrev_b32 %0, 3, %0") }
    if constexpr (OP == 24) { BODY32("v_and_b32 %0, %1, %0") }
    if constexpr (OP == 25) { BODY32("v_mul_f32 %0, %1, %0") }
    if constexpr (OP == 26) { BODY32("v_sub_u32 %0, %1, %0") }
    if constexpr (OP == 27) {
#pragma unroll
      for (int c = 0; c < CH; ++c) { uint64_t cy; asm volatile("v_mad_i64_i32 %0, %1, %2, %3, %0" : "+v"(q[c]), "=s"(cy) : "v"(a), "v"(b)); }
    }
    if constexpr (OP == 28) {
#pragma unroll
      for (int c = 0; c < CH; ++c) asm volatile("v_ashrrev_i64 %0, 7, %0" : "+v"(q[c]));
    }
    if constexpr (OP == 29) {  // dependent mad chain, 1 chain per lane (latency)
      uint64_t cy; asm volatile("v_mad_i64_i32 %0, %1, %2, %3, %0" : "+v"(q[0]), "=s"(cy) : "v"(a), "v"(b));
    }
    if constexpr (OP == 30) { BODY32("v_cndmask_b32 %0, %1, %0, vcc") }
    if constexpr (OP == 31) {
#pragma unroll
      for (int c = 0; c < CH; ++c) asm volatile("v_mov_b64 %0, %1" : "=v"(q[c]) : "v"(q[(c + 1) % CH]));
    }
  }
  uint32_t acc = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) acc += r[c] + (uint32_t)q[c] + (uint32_t)(q[c] >> 32) + (uint32_t)d[c];
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

static const char* NAMES[] = {"v_add_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_mul_u32_u24", "v_mul_hi_u32_u24",
                              "v_mad_u32_u24", "v_mad_u64_u32(+carry)", "v_fma_f64", "v_dot2_u32_u16", "v_lshl_add_u64",
                              "v_add3_u32", "v_alignbit_b32", "v_add_co+v_addc_co (2 instr)", "v_lshrrev_b64",
                              "v_bfe_u32", "u64 a*b+q (compiler)", "v_mad_u32_u16", "v_lshl_add_u32", "v_xor_b32", "v_add_u32_e64", "v_fma_f32", "v_pk_fma_f32",
                              "v_add_co_u32", "v_lshlrev_b32", "v_and_b32", "v_mul_f32", "v_sub_u32", "v_mad_i64_i32", "v_ashrrev_i64", "mad_i64 dependent (1 chain)", "v_cndmask_b32", "v_mov_b64"};

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
  double n = (double)blocks * 256 * ITERS * (OP == 29 ? 1 : CH) * (OP == 12 ? 2 : 1);
  double rate = n / (best * 1e-3);
  // full rate reference: 256 CU x 128 lanes/clk x 2.4 GHz
  printf("%-30s %8.3f ms  %8.2f Tlane-op/s  (%.3f of 7.86e13 full-rate)\n", NAMES[OP], best, rate / 1e12,
         rate / 7.864e13);
  return 0;
}

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  printf("device %s CUs=%d clock=%d kHz\n", p.gcnArchName, p.multiProcessorCount, p.clockRate);
  int blocks = p.multiProcessorCount * 8;  // 8 waves/SIMD-group... 2048 threads per CU
  uint32_t* dout;
  CHECK(hipMalloc(&dout, (size_t)blocks * 256 * 4));
  run<0>(dout, blocks); run<1>(dout, blocks); run<2>(dout, blocks); run<3>(dout, blocks);
  run<4>(dout, blocks); run<5>(dout, blocks); run<6>(dout, blocks); run<7>(dout, blocks);
  run<8>(dout, blocks); run<9>(dout, blocks); run<10>(dout, blocks); run<11>(dout, blocks);
  run<12>(dout, blocks); run<13>(dout, blocks); run<14>(dout, blocks); run<15>(dout, blocks);
  run<16>(dout, blocks); run<17>(dout, blocks); run<18>(dout, blocks); run<19>(dout, blocks);
  run<20>(dout, blocks); run<21>(dout, blocks); run<22>(dout, blocks); run<23>(dout, blocks);
  run<24>(dout, blocks); run<25>(dout, blocks); run<26>(dout, blocks);
  run<27>(dout, blocks); run<28>(dout, blocks); run<30>(dout, blocks); run<31>(dout, blocks);
  printf("-- 1 wave/SIMD, 1 dependent chain --\n");
  run<29>(dout, blocks/8);
  printf("-- at 4 waves/SIMD --\n");
  run<0>(dout, blocks/2); run<6>(dout, blocks/2); run<10>(dout, blocks/2); run<20>(dout, blocks/2);
  printf("-- at 1 wave/SIMD --\n");
  run<0>(dout, blocks/8); run<6>(dout, blocks/8); run<10>(dout, blocks/8); run<20>(dout, blocks/8);
  CHECK(hipFree(dout));
  return 0;
}
