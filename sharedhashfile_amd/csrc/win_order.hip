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
// Three launches, one workgroup per chunk of kWoChunk keys:
//   k_wo_rank        (shf_win_order*) the chunk's stable order by window from
//                    its 16-B hash records (win_rank.h: ballot ranks per wave,
//                    scans per window), written as 4096 u16 key offsets, and its
//                    256 window counts into the bin-major counts; or
//                    k_wo_rank_bytes, the same from the window bytes a hashing
//                    kernel wrote beside its records (shf_hash_batch_*_win*,
//                    kOutHashWin; 1 B per key) -- or nothing, when the 16-B
//                    hashing kernel ranked the chunks itself (k_fixed16_win);
//   k_wo_scan_rows   the bin-major counts scanned per window, one row each;
//   k_wo_place       each key of the chunk's order written to its place in perm.
// Ranking where the windows are already in registers leaves the launch after
// the scan one load and one store per key.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/shf_hash_batch.h"
#include "kernels.h"
#include "win_rank.h"

namespace shfhb {

namespace {

constexpr uint32_t kWoThreads = 256;                 // 4 waves
constexpr uint32_t kWoSteps = kWoChunk / kWoThreads;  // keys per lane (steps of 64 keys per wave)
static_assert(kWoChunk == 4096 && kWoBins == 256, "one chunk = 4 waves x 16 steps x 64 keys; one window per thread");

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));


// One chunk per workgroup, its order by window from the 16-B hash records (h1's
// low byte, shf.c:800): the sixteen record loads of a lane in flight before the
// first is used (past the batch: the last key's record, ranked nowhere).
__global__ __launch_bounds__(kWoThreads) void k_wo_rank(const u32x4* __restrict__ hashes, uint64_t n,
                                                       uint32_t* __restrict__ counts, uint16_t* __restrict__ sorted) {
  __shared__ WoRankLds<kWoThreads / 64> L;
  const uint32_t t = threadIdx.x, wave = t >> 6, lane = t & 63u;
  const uint32_t c = xcd_major(blockIdx.x, gridDim.x);
  const uint64_t k0 = (uint64_t)c * kWoChunk;
  const uint32_t kn = (uint32_t)min<uint64_t>(kWoChunk, n - k0);
  wo_rank_init(L);
  uint32_t w[kWoSteps];
#pragma unroll
  for (uint32_t q = 0; q < kWoSteps; ++q)
    w[q] = __builtin_nontemporal_load(&hashes[k0 + min(wo_key_of<kWoSteps>(wave, q, lane), kn - 1u)]).x & 0xffu;
  wo_rank_chunk<kWoThreads / 64, kWoSteps>(w, kn, L, counts + c, wo_row_stride(gridDim.x), sorted + k0);
}

// The same from the window bytes a hashing kernel wrote (kOutHashWin): 1 B per
// key read instead of the 16-B record (the workspace holds whole chunks; bytes
// past the batch are ranked nowhere).
__global__ __launch_bounds__(kWoThreads) void k_wo_rank_bytes(const uint8_t* __restrict__ wins, uint64_t n,
                                                             uint32_t* __restrict__ counts,
                                                             uint16_t* __restrict__ sorted) {
  __shared__ WoRankLds<kWoThreads / 64> L;
  const uint32_t t = threadIdx.x, wave = t >> 6, lane = t & 63u;
  const uint32_t c = xcd_major(blockIdx.x, gridDim.x);
  const uint64_t k0 = (uint64_t)c * kWoChunk;
  const uint32_t kn = (uint32_t)min<uint64_t>(kWoChunk, n - k0);
  wo_rank_init(L);
  uint32_t w[kWoSteps];
#pragma unroll
  for (uint32_t q = 0; q < kWoSteps; ++q) w[q] = __builtin_nontemporal_load(&wins[k0 + wo_key_of<kWoSteps>(wave, q, lane)]);
  wo_rank_chunk<kWoThreads / 64, kWoSteps>(w, kn, L, counts + c, wo_row_stride(gridDim.x), sorted + k0);
}

// The chunks' counts scanned per bin in one launch: one workgroup per bin
// scans its row (bin-major counts: the row is contiguous), 16 consecutive
// chunks per thread (four 16-B loads) and 4096 per pass, and writes the
// exclusive prefix back in place, then the bin's total at entry [chunks].
__global__ __launch_bounds__(256) void k_wo_scan_rows(uint32_t* __restrict__ counts, uint32_t chunks) {
  constexpr uint32_t kPer = 16;
  __shared__ uint32_t wsum[4];
  const uint32_t t = threadIdx.x, lane = t & 63u, wave = t >> 6;
  uint32_t* row = counts + (uint64_t)blockIdx.x * wo_row_stride(chunks);
  uint32_t carry = 0;
  for (uint32_t c0 = 0; c0 < chunks; c0 += 256u * kPer) {
    const uint32_t cb = c0 + kPer * t;  // this thread's first chunk (16-B aligned: c0 and kPer are)
    uint32_t v[kPer];
#pragma unroll
    for (uint32_t q = 0; q < kPer / 4; ++q) {
      const u32x4 x = cb + 4u * q < chunks ? *reinterpret_cast<const u32x4*>(row + cb + 4u * q) : u32x4{0, 0, 0, 0};
      v[4 * q] = x.x, v[4 * q + 1] = x.y, v[4 * q + 2] = x.z, v[4 * q + 3] = x.w;
    }
#pragma unroll
    for (uint32_t j = 0; j < kPer; ++j)
      if (cb + j >= chunks) v[j] = 0;  // a 16-B load may reach past the last chunk (the row's slack)
    uint32_t sum = 0;
#pragma unroll
    for (uint32_t j = 0; j < kPer; ++j) sum += v[j];
    const uint32_t inc = wo_wave_incl_scan(sum);  // inclusive scan of the threads' sums over the wave
    if (lane == 63) wsum[wave] = inc;
    __syncthreads();
    uint32_t run = carry + inc - sum, block = 0;
#pragma unroll
    for (uint32_t w = 0; w < 4; ++w) {
      run += w < wave ? wsum[w] : 0u;
      block += wsum[w];
    }
#pragma unroll
    for (uint32_t q = 0; q < kPer / 4; ++q) {
      u32x4 x;
      x.x = run, run += v[4 * q];
      x.y = run, run += v[4 * q + 1];
      x.z = run, run += v[4 * q + 2];
      x.w = run, run += v[4 * q + 3];
      if (cb + 4u * q + 3u < chunks) {
        *reinterpret_cast<u32x4*>(row + cb + 4u * q) = x;
      } else {
        if (cb + 4u * q < chunks) row[cb + 4u * q] = x.x;
        if (cb + 4u * q + 1u < chunks) row[cb + 4u * q + 1u] = x.y;
        if (cb + 4u * q + 2u < chunks) row[cb + 4u * q + 2u] = x.z;
      }
    }
    carry += block;
    __syncthreads();  // wsum is rewritten by the next pass
  }
  if (t == 0) row[chunks] = carry;
}

// One chunk per workgroup, its order (k_wo_rank*) placed: thread b (window b)
// takes the chunk's count of window b (the difference of two scanned entries)
// and the batch total; exclusive scans over the windows give the window's base
// in perm and its first position in the chunk's order; gdelta = their
// difference + the chunk's prefix (k_wo_scan_rows). Thread b marks positions
// [first, first + count) as window b's; then position j of the order goes to
// perm[gdelta[window of j] + j] (thread t the positions t, t + 512, ...: a
// window's keys are consecutive both in the order and in perm, so each store
// instruction writes a few runs of whole lines). The order's entries are loaded
// first, their latency under the scans. 512 threads (threads b < 256 do the
// per-window work): 16.6 us per 10M keys against 17.3 with 256.
constexpr uint32_t kWoPlaceThreads = 512;

__global__ __launch_bounds__(kWoPlaceThreads) void k_wo_place(const uint16_t* __restrict__ sorted, uint64_t n,
                                                             const uint32_t* __restrict__ counts,
                                                             uint32_t* __restrict__ perm,
                                                             uint32_t* __restrict__ win_start) {
  constexpr uint32_t kPer = kWoChunk / kWoPlaceThreads;
  __shared__ uint32_t gdelta[kWoBins];  // window t's perm position minus its position in the chunk's order
  __shared__ __attribute__((aligned(16))) uint8_t win_at[kWoChunk];  // the window of each position of the order
  __shared__ uint32_t tsum[2][4];
  const uint32_t t = threadIdx.x, wave = t >> 6, lane = t & 63u;
  const uint32_t c = xcd_major(blockIdx.x, gridDim.x);
  const uint64_t k0 = (uint64_t)c * kWoChunk;
  const uint32_t kn = (uint32_t)min<uint64_t>(kWoChunk, n - k0);
  uint32_t e[kPer];
#pragma unroll
  for (uint32_t q = 0; q < kPer; ++q) e[q] = sorted[k0 + t + kWoPlaceThreads * q];  // whole chunks in the workspace
  uint32_t tot = 0, pre = 0, hc = 0, it = 0, ih = 0;
  if (t < kWoBins) {
    const uint32_t* row = counts + (uint64_t)t * wo_row_stride(gridDim.x);
    tot = row[gridDim.x];
    pre = row[c];
    hc = row[c + 1] - pre;  // entry [chunks] is the total: the last chunk's difference holds too
    it = wo_wave_incl_scan(tot);
    ih = wo_wave_incl_scan(hc);
    if (lane == 63) {
      tsum[0][wave] = it;
      tsum[1][wave] = ih;
    }
  }
  __syncthreads();
  if (t < kWoBins) {
    uint32_t bbase = it - tot, lbase = ih - hc;
    for (uint32_t v = 0; v < wave; ++v) {
      bbase += tsum[0][v];
      lbase += tsum[1][v];
    }
    if (c == 0 && win_start) {
      win_start[t] = bbase;
      if (t == kWoBins - 1) win_start[kWoBins] = bbase + tot;  // = n
    }
    gdelta[t] = bbase + pre - lbase;
    uint32_t j = lbase;
    const uint32_t je = lbase + hc;
    for (; j < je && (j & 3u); ++j) win_at[j] = (uint8_t)t;
    for (; j + 4u <= je; j += 4u) *reinterpret_cast<uint32_t*>(win_at + j) = t * 0x01010101u;
    for (; j < je; ++j) win_at[j] = (uint8_t)t;
  }
  __syncthreads();
#pragma unroll
  for (uint32_t q = 0; q < kPer; ++q) {
    const uint32_t j = t + kWoPlaceThreads * q;
    const uint32_t at = gdelta[win_at[j]] + j;
    if (j < kn && at < n) perm[at] = (uint32_t)(k0 + e[q]);  // at < n always, unless the counts were not this batch's
  }
}

}  // namespace

// Workspace: the counts (bin-major rows, wo_row_stride), the window bytes
// (whole chunks), then the chunks' orders (4096 u16 per chunk); 16-B aligned
// parts (the rows are whole multiples of 256 B, the chunks of 4 KiB).
uint64_t win_order_workspace_bytes(uint64_t n) {
  const uint64_t chunks = (n + kWoChunk - 1) / kWoChunk;
  return kWoBins * wo_row_stride(chunks) * sizeof(uint32_t) + chunks * kWoChunk * (1 + sizeof(uint16_t));
}

uint32_t* win_order_counts(void* workspace) { return static_cast<uint32_t*>(workspace); }

uint8_t* win_order_wins(void* workspace, uint64_t n) {
  const uint64_t chunks = (n + kWoChunk - 1) / kWoChunk;
  return reinterpret_cast<uint8_t*>(win_order_counts(workspace) + kWoBins * wo_row_stride(chunks));
}

uint16_t* win_order_sorted(void* workspace, uint64_t n) {
  const uint64_t chunks = (n + kWoChunk - 1) / kWoChunk;
  return reinterpret_cast<uint16_t*>(win_order_wins(workspace, n) + chunks * kWoChunk);
}

// The scan and the placement over counts and chunk orders already in the
// workspace (ranked), or after ranking the window bytes.
hipError_t launch_win_order_bytes(uint64_t n, bool ranked, uint32_t* perm, uint32_t* win_start, void* workspace,
                                  hipStream_t st) {
  if (n == 0) {
    if (win_start) return hipMemsetAsync(win_start, 0, (kWoBins + 1) * sizeof(uint32_t), st);
    return hipSuccess;
  }
  if (n > 0xffffffffull) return hipErrorInvalidValue;  // 32-bit key indices
  const uint32_t chunks = (uint32_t)((n + kWoChunk - 1) / kWoChunk);
  uint32_t* counts = win_order_counts(workspace);
  uint16_t* sorted = win_order_sorted(workspace, n);
  if (!ranked)
    hipLaunchKernelGGL(k_wo_rank_bytes, dim3(chunks), dim3(kWoThreads), 0, st, win_order_wins(workspace, n), n,
                       counts, sorted);
  hipLaunchKernelGGL(k_wo_scan_rows, dim3(kWoBins), dim3(256), 0, st, counts, chunks);
  hipLaunchKernelGGL(k_wo_place, dim3(chunks), dim3(kWoPlaceThreads), 0, st, sorted, n, counts, perm, win_start);
  return hipGetLastError();
}

hipError_t launch_win_order(const void* hashes, uint64_t n, uint32_t* perm, uint32_t* win_start, void* workspace,
                            hipStream_t st) {
  if (n == 0 || n > 0xffffffffull) return launch_win_order_bytes(n, true, perm, win_start, workspace, st);
  const uint32_t chunks = (uint32_t)((n + kWoChunk - 1) / kWoChunk);
  hipLaunchKernelGGL(k_wo_rank, dim3(chunks), dim3(kWoThreads), 0, st, static_cast<const u32x4*>(hashes), n,
                     win_order_counts(workspace), win_order_sorted(workspace, n));
  return launch_win_order_bytes(n, true, perm, win_start, workspace, st);
}

}  // namespace shfhb
