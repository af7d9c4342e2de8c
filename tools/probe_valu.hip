// Microbenchmark: issue rate of the integer VALU instructions the Murmur3 kernels
// lower to, on gfx950. Each kernel runs 8 independent chains of one instruction
// per lane in a loop; we report wave-instructions per cycle per CU from wall time
// at the measured clock (s_memtime ticks vs s_memrealtime at 100 MHz).
//
//   hipcc --offload-arch=gfx950 -O3 tools/probe_valu.hip -o tools/probe_valu && ./tools/probe_valu
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e = (x);                                                           \
    if (e != hipSuccess) {                                                        \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

constexpr int kIters = 4096;

#define OP8(INS)                                                                           \
  asm volatile(INS " %0, %0, %8\n\t" INS " %1, %1, %8\n\t" INS " %2, %2, %8\n\t" INS        \
               " %3, %3, %8\n\t" INS " %4, %4, %8\n\t" INS " %5, %5, %8\n\t" INS " %6, %6, %8\n\t" INS \
               " %7, %7, %8"                                                               \
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)  \
               : "v"(k))

template <int OP>
__global__ void k_probe(uint32_t* out, uint32_t seed, unsigned long long* ticks) {
  uint32_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
           a6 = a0 + 6, a7 = a0 + 7;
  const uint32_t k = seed | 1u;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < kIters; ++i) {
    if constexpr (OP == 0) OP8("v_add_u32");
    if constexpr (OP == 1) OP8("v_mul_lo_u32");
    if constexpr (OP == 2) OP8("v_mul_hi_u32");
    if constexpr (OP == 3) OP8("v_xor_b32");
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) *ticks = t1 - t0;
}

// v_mad_u64_u32 (64-bit result) and v_lshl_add_u64 need 64-bit register pairs.
template <int OP>
__global__ void k_probe64(uint64_t* out, uint32_t seed, unsigned long long* ticks) {
  uint64_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
           a6 = a0 + 6, a7 = a0 + 7;
  const uint32_t k = seed | 1u;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < kIters; ++i) {
    if constexpr (OP == 0) {
#define MAD(x) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(x) : "v"(k), "v"(seed) : "vcc")
      MAD(a0); MAD(a1); MAD(a2); MAD(a3); MAD(a4); MAD(a5); MAD(a6); MAD(a7);
    }
    if constexpr (OP == 1) {
#define LSA(x) asm volatile("v_lshl_add_u64 %0, %0, 2, %0" : "+v"(x))
      LSA(a0); LSA(a1); LSA(a2); LSA(a3); LSA(a4); LSA(a5); LSA(a6); LSA(a7);
    }
    if constexpr (OP == 2) {
#define AB(x) asm volatile("v_alignbit_b32 %0, %0, %1, 31" : "+v"(x) : "v"(k))
      uint32_t* p0 = (uint32_t*)&a0;
      uint32_t b0 = p0[0], b1 = (uint32_t)a1, b2 = (uint32_t)a2, b3 = (uint32_t)a3, b4 = (uint32_t)a4,
               b5 = (uint32_t)a5, b6 = (uint32_t)a6, b7 = (uint32_t)a7;
      AB(b0); AB(b1); AB(b2); AB(b3); AB(b4); AB(b5); AB(b6); AB(b7);
      a0 = b0; a1 = b1; a2 = b2; a3 = b3; a4 = b4; a5 = b5; a6 = b6; a7 = b7;
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && blockIdx.x == 0) *ticks = t1 - t0;
}

template <typename K, typename T>
static int run(const char* name, K kern, T* d_out, unsigned long long* d_ticks, int blocks, int threads) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, d_out, 12345u, d_ticks);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, d_out, 12345u, d_ticks);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  unsigned long long ticks = 0;
  CHECK(hipMemcpy(&ticks, d_ticks, sizeof(ticks), hipMemcpyDeviceToHost));
  const double waves = (double)blocks * threads / 64.0;
  const double wave_instr = waves * kIters * 8.0;
  const double lane_ops_per_s = wave_instr * 64.0 / (ms * 1e-3);
  // one wave's own cycles per instruction (s_memtime ticks at shader clock)
  printf("%-16s %8.3f ms  %8.2f T lane-ops/s  %6.2f cyc/instr (1 wave, loaded chip)\n", name, ms,
         lane_ops_per_s / 1e12, (double)ticks / (kIters * 8.0));
  return 0;
}

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  printf("device %s, %d CUs, clock %d kHz\n", p.gcnArchName, p.multiProcessorCount, p.clockRate);
  const int threads = 256, blocks = p.multiProcessorCount * 8;
  uint32_t* d32;
  uint64_t* d64;
  unsigned long long* dt;
  CHECK(hipMalloc(&d32, (size_t)blocks * threads * 4));
  CHECK(hipMalloc(&d64, (size_t)blocks * threads * 8));
  CHECK(hipMalloc(&dt, 8));
  run("v_add_u32", k_probe<0>, d32, dt, blocks, threads);
  run("v_xor_b32", k_probe<3>, d32, dt, blocks, threads);
  run("v_mul_lo_u32", k_probe<1>, d32, dt, blocks, threads);
  run("v_mul_hi_u32", k_probe<2>, d32, dt, blocks, threads);
  run("v_mad_u64_u32", k_probe64<0>, d64, dt, blocks, threads);
  run("v_lshl_add_u64", k_probe64<1>, d64, dt, blocks, threads);
  run("v_alignbit_b32", k_probe64<2>, d64, dt, blocks, threads);
  return 0;
}
