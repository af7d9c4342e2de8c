// Window order of a batch (SURVEY.md §8 f1's stated use: "sorting a batch by
// win"): a stable counting sort of the batch's key indices by the window their
// hash selects, win = h1 & 0xff (/root/reference/src/shf.c:800, :893).
//
// Every structure a put/get/del touches belongs to one window: its lock
// (shf.c:805, :904), its tab2 -> tab map, its tabs and their files (a new tab
// is numbered by the window's own tabs_used, shf.c:432). Keys of different
// windows never interact, so replaying a batch window by window, keeping the
// batch order inside each window, leaves the store exactly as the batch order
// does (tests/test_win_order.py checks the reference's own files and uids), and
// consecutive operations then find the window's lock, map and tabs in cache:
// the reference's get loop runs ~1.5x faster in window order.
//
// Three launches, all HBM-bound (16-B hash records in, 4-B indices out; the
// records are read once: 16 + 1 + 1 + 4 B per key against 20 B at least):
//   k_wo_hist     one wave per chunk of kWoChunk keys, four keys per lane per
//                 step: the chunk's 256-bin histogram (LDS atomics), written
//                 bin-major (counts[bin * chunks + chunk]), and each key's
//                 window as one byte (wins[key]) for the scatter;
//   k_wo_scan     one workgroup per bin: exclusive scan of the bin's chunk
//                 counts in place, the bin's total beside them;
//   k_wo_scatter  one wave per chunk again, in key order, 64 keys per step
//                 (their window bytes, not the records):
//                 the lanes of a step holding the same window find each other
//                 with eight ballots (one per window bit), the lowest takes
//                 the window's next positions for all of them, each lane
//                 writes its key index at base + its rank among them. The
//                 window's running position lives in the wave's LDS (a wave's
//                 LDS accesses execute in order, and the compiler keeps the
//                 order of these aliasing ones: no fence between steps).
// Chunks are numbered XCD by XCD (workgroup g runs on XCD g % 8), so the runs
// of positions that consecutive chunks write into one window's range are
// written through the same L2 and leave HBM as whole lines.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/shf_hash_batch.h"
#include "kernels.h"

namespace shfhb {

namespace {

constexpr uint32_t kWoChunk = 4096;  // keys per chunk = 64 steps of one wave
constexpr uint32_t kWoWaves = 4;     // waves (chunks) per workgroup
constexpr uint32_t kWoBins = 256;    // SHF_WINS_PER_SHF

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Workgroup g's place in XCD-major order: the g % 8 == x workgroups of a launch
// (those on XCD x) take consecutive slots.
__device__ __forceinline__ uint32_t xcd_major(uint32_t g, uint32_t groups) {
  const uint32_t q = groups / 8u, r = groups % 8u, x = g % 8u;
  return x * q + min(x, r) + g / 8u;
}

__device__ __forceinline__ uint32_t win_of(const u32x4* hashes, uint64_t key) {
  return __builtin_nontemporal_load(&hashes[key]).x & 0xffu;  // h1's low byte (shf.c:800)
}

__global__ __launch_bounds__(64 * kWoWaves) void k_wo_hist(const u32x4* __restrict__ hashes, uint64_t n,
                                                          uint32_t chunks, uint32_t* __restrict__ counts,
                                                          uint32_t* __restrict__ wins) {
  __shared__ uint32_t hist[kWoWaves][kWoBins];
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const uint32_t c = xcd_major(blockIdx.x, gridDim.x) * kWoWaves + wave;
  for (uint32_t b = lane; b < kWoBins; b += 64u) hist[wave][b] = 0;
  if (c >= chunks) return;
  const uint64_t k0 = (uint64_t)c * kWoChunk;
  const uint32_t kn = (uint32_t)min<uint64_t>(kWoChunk, n - k0);
  // step: 256 keys, lane l the four at 4 l (64 B of records, one u32 of window bytes)
#pragma unroll 2
  for (uint32_t i0 = 0; i0 < kn; i0 += 256u) {
    const uint32_t i = i0 + 4u * lane;
    uint32_t packed = 0;
#pragma unroll
    for (uint32_t q = 0; q < 4u; ++q)
      if (i + q < kn) {
        const uint32_t w = win_of(hashes, k0 + i + q);
        atomicAdd(&hist[wave][w], 1u);
        packed |= w << (8u * q);
      }
    if (i < kn) wins[(k0 + i) >> 2] = packed;  // kWoChunk is a multiple of 4: k0 + i is too
  }
  for (uint32_t b = lane; b < kWoBins; b += 64u) counts[(uint64_t)b * chunks + c] = hist[wave][b];
}

// Exclusive scan of one bin's chunk counts, in place; totals[bin] = the sum.
__global__ __launch_bounds__(256) void k_wo_scan(uint32_t* __restrict__ counts, uint32_t chunks,
                                                 uint32_t* __restrict__ totals) {
  __shared__ uint32_t wsum[4];
  uint32_t* row = counts + (uint64_t)blockIdx.x * chunks;
  const uint32_t t = threadIdx.x, lane = t & 63u, wave = t >> 6;
  uint32_t carry = 0;
  for (uint32_t base = 0; base < chunks; base += 1024u) {
    // four consecutive counts per thread
    uint32_t v[4], s = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t i = base + 4u * t + j;
      v[j] = i < chunks ? row[i] : 0u;
      s += v[j];
    }
    uint32_t incl = s;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
      const uint32_t u = (uint32_t)__shfl_up((int)incl, d);
      if (lane >= d) incl += u;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint32_t before = carry;
    for (uint32_t w = 0; w < wave; ++w) before += wsum[w];
    const uint32_t tile = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
    uint32_t run = before + incl - s;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t i = base + 4u * t + j;
      if (i < chunks) row[i] = run;
      run += v[j];
    }
    carry += tile;
  }
  if (t == 0) totals[blockIdx.x] = carry;
}

__global__ __launch_bounds__(64 * kWoWaves) void k_wo_scatter(const uint8_t* __restrict__ wins, uint64_t n,
                                                             uint32_t chunks, const uint32_t* __restrict__ counts,
                                                             const uint32_t* __restrict__ totals,
                                                             uint32_t* __restrict__ perm,
                                                             uint32_t* __restrict__ win_start) {
  __shared__ uint32_t next[kWoWaves][kWoBins];  // the window's next position in perm
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const uint32_t c = xcd_major(blockIdx.x, gridDim.x) * kWoWaves + wave;
  if (c >= chunks) return;
  // bin bases: exclusive scan of the 256 totals, four consecutive bins per lane
  uint32_t t4[4], s = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    t4[j] = totals[4u * lane + j];
    s += t4[j];
  }
  uint32_t incl = s;
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t u = (uint32_t)__shfl_up((int)incl, d);
    if (lane >= d) incl += u;
  }
  uint32_t run = incl - s;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t b = 4u * lane + j;
    next[wave][b] = run + counts[(uint64_t)b * chunks + c];
    if (c == 0 && win_start) win_start[b] = run;
    run += t4[j];
  }
  if (c == 0 && win_start && lane == 63) win_start[kWoBins] = run;  // = n
  const uint64_t k0 = (uint64_t)c * kWoChunk;
  const uint32_t kn = (uint32_t)min<uint64_t>(kWoChunk, n - k0);
  uint32_t w_next = lane < kn ? wins[k0 + lane] : 0u;
  for (uint32_t i0 = 0; i0 < kn; i0 += 64u) {
    const uint32_t i = i0 + lane;
    const bool valid = i < kn;
    const uint32_t w = w_next;
    if (i + 64u < kn) w_next = wins[k0 + i + 64u];  // the next step's window, in flight meanwhile
    if (valid) {
      // lanes of this step holding window w (valid lanes only: ballots see active lanes)
      uint64_t peers = __ballot(1);  // the valid lanes
#pragma unroll
      for (uint32_t bit = 0; bit < 8u; ++bit) {
        const bool set = (w >> bit) & 1u;
        const uint64_t m = __ballot(set);
        peers &= set ? m : ~m;
      }
      const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(peers >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)peers, 0u));
      const uint32_t base = next[wave][w];
      perm[base + rank] = (uint32_t)(k0 + i);
      if (rank == 0) next[wave][w] = base + (uint32_t)__popcll(peers);  // one lane per window: no conflict
    }
  }
}

}  // namespace

uint64_t win_order_workspace_bytes(uint64_t n) {  // counts, totals, then the window bytes
  const uint64_t chunks = (n + kWoChunk - 1) / kWoChunk;
  return (chunks * kWoBins + kWoBins) * sizeof(uint32_t) + ((n + 15u) & ~(uint64_t)15);
}

hipError_t launch_win_order(const void* hashes, uint64_t n, uint32_t* perm, uint32_t* win_start, void* workspace,
                            hipStream_t st) {
  if (n == 0) {
    if (win_start) return hipMemsetAsync(win_start, 0, (kWoBins + 1) * sizeof(uint32_t), st);
    return hipSuccess;
  }
  if (n > 0xffffffffull) return hipErrorInvalidValue;  // 32-bit key indices
  const uint32_t chunks = (uint32_t)((n + kWoChunk - 1) / kWoChunk);
  const uint32_t groups = (chunks + kWoWaves - 1) / kWoWaves;
  uint32_t* counts = static_cast<uint32_t*>(workspace);
  uint32_t* totals = counts + (uint64_t)chunks * kWoBins;
  uint32_t* wins = totals + kWoBins;  // 16-B aligned: the counts are whole chunks of 256 u32
  const u32x4* h = static_cast<const u32x4*>(hashes);
  hipLaunchKernelGGL(k_wo_hist, dim3(groups), dim3(64 * kWoWaves), 0, st, h, n, chunks, counts, wins);
  hipLaunchKernelGGL(k_wo_scan, dim3(kWoBins), dim3(256), 0, st, counts, chunks, totals);
  hipLaunchKernelGGL(k_wo_scatter, dim3(groups), dim3(64 * kWoWaves), 0, st, reinterpret_cast<const uint8_t*>(wins),
                     n, chunks, counts, totals, perm, win_start);
  return hipGetLastError();
}

}  // namespace shfhb
