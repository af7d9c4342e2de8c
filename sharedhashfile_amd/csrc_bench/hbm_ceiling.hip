// Measurement kernels: the HBM ceilings bench.py divides the hashing kernels'
// rates by, measured on the same box in the same run (include/shf_hash_batch_ceiling.h).
// Built into its own library, libshf_hb_bench.so, which only bench.py, tools/ and
// the tests load: the product library libshf_hash_batch.so does not contain or
// export them. Not part of the hashing path: each kernel moves exactly the bytes of one
// hashing kernel's access pattern and computes nothing but an XOR fold.
//
//   k_ceil_copy      lane i: one 16-B nontemporal load of src[i], one 16-B store
//                    to dst[i]; 256-thread blocks, one lane per 16 B -- k_fixed16's
//                    shape (configs[1]) without the hash. 32 B per lane.
//   k_ceil_copy4     the same bytes, 4 x 16 B per lane (a block copies 1024
//                    consecutive 16-B units, lane l units l, l + 256, ...): more
//                    loads in flight per wave than k_fixed16's shape allows.
//   k_ceil_read16    lane i: 16 x 16-B nontemporal loads (its wave reads one
//                    contiguous 16-KiB span, 1 KiB per instruction, the way k_tiled
//                    and k_span stage a tile), their XOR stored as 16 B. 272 B per
//                    lane: configs[2]'s 256 + 16 B per key (configs[3]: 284).
//                    Plain or nontemporal store (the hashing kernels store nt);
//                    256-thread workgroups, or one wave per workgroup (k_tiled's
//                    and k_span's launch shape).
//   k_ceil_gather128 lane i: one 128-B row rows[idx[i]] (the row index read as a
//                    4-B stream), fetched 8 lanes per row exactly as the probe's
//                    row fetch does (probe_scan_coop), 16 B stored per lane. With
//                    idx a permutation every row is read once: 148 B per lane.
//   k_ceil_stream16u lane i: one 16-B load at src + 16 i + shift (shift 1..15:
//                    byte-unaligned, as the tab copy's record gathers load), one
//                    16-B store to dst[i]. 32 B per lane, each source line read
//                    once (a calibration of FETCH_SIZE for unaligned loads).
//   k_ceil_valu<MUL> no memory traffic but one 16-B store per lane: 8
//                    independent chains of v_add_u32 (MUL = 0) or v_mul_lo_u32
//                    (MUL = 1) per lane, `iters` rounds -- a VALU-saturating
//                    launch, to read what rocprof's VALUBusy formula reports for
//                    a SIMD that is busy every cycle with full-rate or with
//                    half-rate instructions (tools/probe_valu.hip's rates).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/shf_hash_batch_ceiling.h"

namespace shfhb {
namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4_a1 __attribute__((ext_vector_type(4), aligned(1)));
typedef __attribute__((address_space(1))) const u32x4 g_u32x4;
typedef __attribute__((address_space(1))) const u32x4_a1 g_u32x4_a1;

constexpr uint32_t kBlock = 256;

__global__ __launch_bounds__(kBlock) void k_ceil_copy(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                      uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  dst[i] = __builtin_nontemporal_load(&src[i]);
}

// Variants of the one-lane-per-16-B copy (tools/copy_sweep.py picks the best for bench.py):
// V = 0 plain loads, 1 nt loads + nt stores, 2 nt loads + s_sleep between load and store (the hash's
// delay: reads and writes of a wave further apart), 3 two units per lane (block-strided)
template <int V>
__global__ __launch_bounds__(kBlock) void k_ceil_copyv(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                       uint64_t n) {
  if constexpr (V == 3) {
    const uint64_t i0 = (uint64_t)blockIdx.x * (2 * kBlock) + threadIdx.x;
    u32x4 a = {0u, 0u, 0u, 0u}, b = {0u, 0u, 0u, 0u};
    if (i0 < n) a = __builtin_nontemporal_load(&src[i0]);
    if (i0 + kBlock < n) b = __builtin_nontemporal_load(&src[i0 + kBlock]);
    if (i0 < n) dst[i0] = a;
    if (i0 + kBlock < n) dst[i0 + kBlock] = b;
    return;
  }
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  if constexpr (V == 0) {
    dst[i] = src[i];
  } else if constexpr (V == 1) {
    __builtin_nontemporal_store(__builtin_nontemporal_load(&src[i]), &dst[i]);
  } else {
    const u32x4 v = __builtin_nontemporal_load(&src[i]);
    __builtin_amdgcn_s_sleep(3);
    dst[i] = v;
  }
}

__global__ __launch_bounds__(kBlock) void k_ceil_copy4(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                       uint64_t n) {
  const uint64_t i0 = (uint64_t)blockIdx.x * (4 * kBlock) + threadIdx.x;
  u32x4 v[4];
#pragma unroll
  for (uint32_t q = 0; q < 4; ++q)
    if (i0 + q * kBlock < n) v[q] = __builtin_nontemporal_load(&src[i0 + q * kBlock]);
#pragma unroll
  for (uint32_t q = 0; q < 4; ++q)
    if (i0 + q * kBlock < n) dst[i0 + q * kBlock] = v[q];
}

template <bool NT_STORE, uint32_t BLOCK = kBlock>
__global__ __launch_bounds__(BLOCK) void k_ceil_read16(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                       uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  const uint64_t wave = i >> 6;
  const uint32_t lane = threadIdx.x & 63u;
  if (wave * 64u >= n) return;  // whole waves only: n is a multiple of 64 (checked by the launcher)
  const u32x4* span = src + wave * 64u * 16u;
  u32x4 v[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) v[q] = __builtin_nontemporal_load(&span[64 * q + lane]);
  u32x4 x = v[0];
#pragma unroll
  for (int q = 1; q < 16; ++q) x ^= v[q];
  if constexpr (NT_STORE) __builtin_nontemporal_store(x, &dst[i]);
  else dst[i] = x;
}

// IDX16: the index arrives as 16-B records (the row index in the first word), as
// the probe reads a 16-B key per lane, and the result is stored nontemporally as
// the probe stores its record: SHF_HB_CEIL_PROBE_ROWS, 160 B per lane.
// An index naming a row past n_rows reads row 0 instead (never past src).
template <bool IDX16>
__global__ __launch_bounds__(kBlock) void k_ceil_gather128(const uint8_t* __restrict__ rows, uint32_t n_rows,
                                                           const uint32_t* __restrict__ idx, u32x4* __restrict__ dst,
                                                           uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63u;
  uint32_t r = 0;  // lanes past n fetch row 0 and discard it
  if (i < n) {
    if constexpr (IDX16) r = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(idx) + i).x;
    else r = __builtin_nontemporal_load(&idx[i]);
    r = r < n_rows ? r : 0u;
  }
  u32x4 g[8];
#pragma unroll
  for (uint32_t q = 0; q < 8; ++q) {
    const uint32_t rq = (uint32_t)__shfl((int)r, (int)(8u * q + (lane >> 3)));
    g[q] = *reinterpret_cast<g_u32x4*>(reinterpret_cast<uintptr_t>(rows) + ((uint64_t)rq << 7) + 16u * (lane & 7u));
  }
  u32x4 x = g[0];
#pragma unroll
  for (int q = 1; q < 8; ++q) x ^= g[q];
  if (i < n) {
    if constexpr (IDX16) __builtin_nontemporal_store(x, &dst[i]);
    else dst[i] = x;
  }
}

__global__ __launch_bounds__(kBlock) void k_ceil_stream16u(const uint8_t* __restrict__ src, u32x4* __restrict__ dst,
                                                           uint64_t n, uint32_t shift) {
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  dst[i] = *reinterpret_cast<g_u32x4_a1*>(reinterpret_cast<uintptr_t>(src) + 16u * i + shift);
}

#define SHFHB_OP8(INS)                                                                                   \
  asm volatile(INS " %0, %0, %8\n\t" INS " %1, %1, %8\n\t" INS " %2, %2, %8\n\t" INS " %3, %3, %8\n\t" INS \
               " %4, %4, %8\n\t" INS " %5, %5, %8\n\t" INS " %6, %6, %8\n\t" INS " %7, %7, %8"               \
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)          \
               : "v"(k))

template <int MUL>
__global__ __launch_bounds__(kBlock) void k_ceil_valu(uint32_t seed, u32x4* __restrict__ dst, uint64_t n,
                                                      uint32_t iters) {
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  uint32_t a0 = (uint32_t)i ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
           a7 = a0 + 7;
  const uint32_t k = seed | 1u;
  for (uint32_t r = 0; r < iters; ++r) {
    if constexpr (MUL) SHFHB_OP8("v_mul_lo_u32");
    else SHFHB_OP8("v_add_u32");
  }
  if (i < n) dst[i] = u32x4{a0 ^ a1, a2 ^ a3, a4 ^ a5, a6 ^ a7};
}
#undef SHFHB_OP8

}  // namespace
}  // namespace shfhb

extern "C" int shf_hb_ceiling_async(int kind, const void* d_src, uint64_t src_bytes, const uint32_t* d_idx,
                                    void* d_dst, uint64_t n, void* hip_stream) {
  using namespace shfhb;
  if (n == 0) return SHF_HB_OK;
  if (!d_src || !d_dst || (n + kBlock - 1) / kBlock > 0x7fffffffull) return SHF_HB_ERR_ARG;
  if (((uintptr_t)d_dst & 15u) != 0) return SHF_HB_ERR_ARG;
  const dim3 grid((unsigned)((n + kBlock - 1) / kBlock)), block(kBlock);
  const hipStream_t st = (hipStream_t)hip_stream;
  const bool al16 = ((uintptr_t)d_src & 15u) == 0;
  switch (kind) {
    case SHF_HB_CEIL_COPY:
      if (!al16 || src_bytes < 16u * n) return SHF_HB_ERR_ARG;
      hipLaunchKernelGGL(k_ceil_copy, grid, block, 0, st, (const u32x4*)d_src, (u32x4*)d_dst, n);
      break;
    case SHF_HB_CEIL_COPY4:
      if (!al16 || src_bytes < 16u * n) return SHF_HB_ERR_ARG;
      hipLaunchKernelGGL(k_ceil_copy4, dim3((unsigned)((n + 4 * kBlock - 1) / (4 * kBlock))), block, 0, st,
                         (const u32x4*)d_src, (u32x4*)d_dst, n);
      break;
    case SHF_HB_CEIL_COPY_PLAIN:
    case SHF_HB_CEIL_COPY_NT:
    case SHF_HB_CEIL_COPY_SLEEP:
    case SHF_HB_CEIL_COPY2: {
      if (!al16 || src_bytes < 16u * n) return SHF_HB_ERR_ARG;
      const dim3 g2((unsigned)((n + 2 * kBlock - 1) / (2 * kBlock)));
      const u32x4* s4 = (const u32x4*)d_src;
      u32x4* d4 = (u32x4*)d_dst;
      if (kind == SHF_HB_CEIL_COPY_PLAIN) hipLaunchKernelGGL(k_ceil_copyv<0>, grid, block, 0, st, s4, d4, n);
      else if (kind == SHF_HB_CEIL_COPY_NT) hipLaunchKernelGGL(k_ceil_copyv<1>, grid, block, 0, st, s4, d4, n);
      else if (kind == SHF_HB_CEIL_COPY_SLEEP) hipLaunchKernelGGL(k_ceil_copyv<2>, grid, block, 0, st, s4, d4, n);
      else hipLaunchKernelGGL(k_ceil_copyv<3>, g2, block, 0, st, s4, d4, n);
      break;
    }
    case SHF_HB_CEIL_READ16:
    case SHF_HB_CEIL_READ16_NT:
    case SHF_HB_CEIL_READ16_W1:
      if (!al16 || n % 64u || src_bytes < 256u * n) return SHF_HB_ERR_ARG;
      if (kind == SHF_HB_CEIL_READ16)
        hipLaunchKernelGGL(k_ceil_read16<false>, grid, block, 0, st, (const u32x4*)d_src, (u32x4*)d_dst, n);
      else if (kind == SHF_HB_CEIL_READ16_NT)
        hipLaunchKernelGGL(k_ceil_read16<true>, grid, block, 0, st, (const u32x4*)d_src, (u32x4*)d_dst, n);
      else if (n / 64u > 0x7fffffffull)
        return SHF_HB_ERR_ARG;
      else  // one wave per workgroup: k_tiled's launch shape
        hipLaunchKernelGGL((k_ceil_read16<true, 64>), dim3((unsigned)(n / 64u)), dim3(64), 0, st,
                           (const u32x4*)d_src, (u32x4*)d_dst, n);
      break;
    case SHF_HB_CEIL_GATHER128:
    case SHF_HB_CEIL_PROBE_ROWS: {
      // an idx[i] >= src_bytes / 128 is clamped to row 0 by the kernel (the launcher cannot read device memory)
      if (!al16 || !d_idx || src_bytes < 128u || src_bytes / 128u > 0xffffffffull) return SHF_HB_ERR_ARG;
      const uint32_t n_rows = (uint32_t)(src_bytes / 128u);
      if (kind == SHF_HB_CEIL_GATHER128)
        hipLaunchKernelGGL(k_ceil_gather128<false>, grid, block, 0, st, (const uint8_t*)d_src, n_rows, d_idx,
                           (u32x4*)d_dst, n);
      else if ((reinterpret_cast<uintptr_t>(d_idx) & 15u) != 0)
        return SHF_HB_ERR_ARG;
      else  // with the probe kernel's 32 KiB of LDS per 256-thread workgroup, hence its occupancy
        hipLaunchKernelGGL(k_ceil_gather128<true>, grid, block, 32u * 1024u, st, (const uint8_t*)d_src, n_rows,
                           d_idx, (u32x4*)d_dst, n);
      break;
    }
    case SHF_HB_CEIL_STREAM16U: {
      const uint32_t shift = (uint32_t)(((uintptr_t)d_src) & 15u) ? 0u : 7u;  // aligned base: read 7 bytes in
      if (src_bytes < 16u * n + 16u) return SHF_HB_ERR_ARG;
      hipLaunchKernelGGL(k_ceil_stream16u, grid, block, 0, st, (const uint8_t*)d_src, (u32x4*)d_dst, n, shift);
      break;
    }
    case SHF_HB_CEIL_VALU_ADD:
    case SHF_HB_CEIL_VALU_MUL: {
      // d_src is not read; src_bytes is the loop count per lane
      if (src_bytes == 0 || src_bytes > 0xffffffffull) return SHF_HB_ERR_ARG;
      const uint32_t iters = (uint32_t)src_bytes, seed = (uint32_t)(uintptr_t)d_src;
      if (kind == SHF_HB_CEIL_VALU_ADD)
        hipLaunchKernelGGL(k_ceil_valu<0>, grid, block, 0, st, seed, (u32x4*)d_dst, n, iters);
      else
        hipLaunchKernelGGL(k_ceil_valu<1>, grid, block, 0, st, seed, (u32x4*)d_dst, n, iters);
      break;
    }
    default:
      return SHF_HB_ERR_ARG;
  }
  return hipGetLastError() == hipSuccess ? SHF_HB_OK : SHF_HB_ERR_HIP;
}

// The device address of page-locked host memory (bench.py pcie_ceilings: the
// copy kernel run over PCIe, reading and/or writing host memory as the
// product's zero copy does); SHF_HB_ERR_ARG for memory the device cannot map.
extern "C" int shf_hb_host_device_ptr(const void* host, void** dev) {
  if (!host || !dev) return SHF_HB_ERR_ARG;
  *dev = nullptr;
  if (hipHostGetDevicePointer(dev, const_cast<void*>(host), 0) != hipSuccess) {
    (void)hipGetLastError();
    return SHF_HB_ERR_ARG;
  }
  return SHF_HB_OK;
}
