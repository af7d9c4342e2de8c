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
// Four launches, HBM-bound (16-B hash records in, 4-B indices out; the
// records are read once: 16 + 1 + 1 + 4 B per key against 20 B at least), one
// workgroup of four waves per chunk of kWoChunk keys:
//   k_wo_hist     the chunk's 256-bin histogram (LDS atomics) as one row of
//                 counts[chunk][bin], and each key's window as one byte;
//   k_wo_scan_*   the chunks' counts scanned per bin in two levels (blocks of
//                 64 rows, then the blocks' sums), rows read whole;
//   k_wo_scatter  the chunk's window bytes staged in LDS; each wave orders its
//                 quarter, 64 keys per step (see the kernel).
// Chunks are numbered XCD by XCD (workgroup g runs on XCD g % 8), so the runs
// of positions that consecutive chunks write into one window's range are
// written through the same L2 and leave HBM as whole lines.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/shf_hash_batch.h"
#include "kernels.h"

namespace shfhb {

namespace {

constexpr uint32_t kWoThreads = 256;                 // 4 waves
constexpr uint32_t kWoSub = 1024;                    // keys per wave (16 steps of 64) in the scatter
constexpr uint32_t kWoChunk = 4 * kWoSub;            // keys per workgroup (a chunk)
constexpr uint32_t kWoBins = 256;                    // SHF_WINS_PER_SHF

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

// One chunk per workgroup: its 256-bin histogram (LDS atomics) as one row of
// counts[c][*] (one coalesced 1-KiB store) and every key's window as one byte.
// Thread t takes keys 256 s + t of step s (each load instruction reads 1 KiB of
// consecutive records); the window bytes gather in LDS and leave as 16 B per
// thread.
__global__ __launch_bounds__(kWoThreads) void k_wo_hist(const u32x4* __restrict__ hashes, uint64_t n,
                                                       uint32_t* __restrict__ counts, uint32_t* __restrict__ wins) {
  __shared__ uint32_t hist[kWoBins];
  __shared__ uint8_t cwb[kWoChunk];
  const uint32_t t = threadIdx.x;
  const uint32_t c = xcd_major(blockIdx.x, gridDim.x);
  hist[t] = 0;
  __syncthreads();
  const uint64_t k0 = (uint64_t)c * kWoChunk;
  const uint32_t kn = (uint32_t)min<uint64_t>(kWoChunk, n - k0);
  // all sixteen record loads in flight before the first is used (past the batch:
  // the last key's record, counted nowhere -- a load under a branch waits at once)
  uint32_t w[16];
#pragma unroll
  for (uint32_t st = 0; st < 16u; ++st) w[st] = win_of(hashes, k0 + min(256u * st + t, kn - 1u));
#pragma unroll
  for (uint32_t st = 0; st < 16u; ++st) {
    const uint32_t i = 256u * st + t;
    if (i < kn) atomicAdd(&hist[w[st]], 1u);
    cwb[i] = (uint8_t)w[st];
  }
  __syncthreads();
  counts[(uint64_t)c * kWoBins + t] = hist[t];
  // 16 window bytes per thread (bytes past the batch land in the workspace's last chunk, unused)
  reinterpret_cast<u32x4*>(wins + (k0 >> 2))[t] = reinterpret_cast<const u32x4*>(cwb)[t];
}

// The chunks' counts scanned per bin in two levels, rows read whole (a row =
// one chunk's 256 counts, 1 KiB; thread t = bin t):
//   k_wo_scan_blocks  one workgroup per block of kWoScanBlock chunks: exclusive
//                     prefix of each bin over the block's rows, in place, and
//                     the block's sums (bsum[block][bin]);
//   k_wo_scan_top     one workgroup: exclusive prefix of each bin over the
//                     blocks' sums, in place, and the bins' totals.
// A chunk's prefix is then counts[c][bin] + bsum[c / kWoScanBlock][bin].
// (One workgroup per bin reading its column, 4-B words 1 KiB apart: 13.4 us
// per 10M keys.)
constexpr uint32_t kWoScanBlock = 64;
__global__ __launch_bounds__(256) void k_wo_scan_blocks(uint32_t* __restrict__ counts, uint32_t chunks,
                                                        uint32_t* __restrict__ bsum) {
  const uint32_t t = threadIdx.x, c0 = blockIdx.x * kWoScanBlock;
  uint32_t v[kWoScanBlock];
#pragma unroll
  for (uint32_t r = 0; r < kWoScanBlock; ++r)  // every load in flight first (past the end: the last row, unused)
    v[r] = counts[(uint64_t)min(c0 + r, chunks - 1u) * kWoBins + t];
  uint32_t run = 0;
#pragma unroll
  for (uint32_t r = 0; r < kWoScanBlock; ++r) {
    if (c0 + r < chunks) counts[(uint64_t)(c0 + r) * kWoBins + t] = run;
    run += c0 + r < chunks ? v[r] : 0u;
  }
  bsum[(uint64_t)blockIdx.x * kWoBins + t] = run;
}

__global__ __launch_bounds__(256) void k_wo_scan_top(uint32_t* __restrict__ bsum, uint32_t blocks,
                                                     uint32_t* __restrict__ totals) {
  constexpr uint32_t kBatch = 16;
  const uint32_t t = threadIdx.x;
  uint32_t run = 0;
  for (uint32_t b0 = 0; b0 < blocks; b0 += kBatch) {
    uint32_t v[kBatch];
#pragma unroll
    for (uint32_t r = 0; r < kBatch; ++r) v[r] = bsum[(uint64_t)min(b0 + r, blocks - 1u) * kWoBins + t];
#pragma unroll
    for (uint32_t r = 0; r < kBatch; ++r) {
      if (b0 + r < blocks) bsum[(uint64_t)(b0 + r) * kWoBins + t] = run;
      run += b0 + r < blocks ? v[r] : 0u;
    }
  }
  totals[t] = run;
}

// One chunk per workgroup, in two phases. (1) The chunk's stable order in LDS:
// wave v takes keys [1024 v, 1024 v + 1024) in key order, 64 per step; the
// lanes of a step holding the same window find each other through a 64-bit LDS
// mask per window (each sets its bit with an atomic OR -- an OR commutes, so
// the order the LDS unit takes the lanes in does not matter -- then reads the
// mask back), the lowest takes the window's next local positions for all of
// them and clears the mask, and each lane puts its key at local start + its
// rank among them. A window's first local position for wave v = the chunk's
// keys of lower windows + the window's keys in waves 0..v-1 (histograms of the
// chunk's window bytes). (2) The chunk's keys leave in that order, thread t
// the positions t, t + 256, ...: a window's keys are consecutive both in LDS
// and in perm (at the window's base, from the totals, + the chunk's prefix,
// k_wo_scan_*), so each store instruction writes a few runs of whole lines
// instead of one scattered index per lane (eight ballots per step instead of
// the masks, with per-lane scattered stores: 47 us per 10M keys).
// A wave's LDS accesses execute in order, and the compiler keeps the order of
// these aliasing ones: no fence between steps.
__global__ __launch_bounds__(kWoThreads) void k_wo_scatter(const uint8_t* __restrict__ wins, uint64_t n,
                                                          uint32_t chunks, const uint32_t* __restrict__ counts,
                                                          const uint32_t* __restrict__ bsum,
                                                          const uint32_t* __restrict__ totals,
                                                          uint32_t* __restrict__ perm,
                                                          uint32_t* __restrict__ win_start) {
  __shared__ uint32_t next[4][kWoBins];         // per wave: the window's next local position
  __shared__ uint32_t cw[kWoChunk / 4];         // the chunk's window bytes
  __shared__ uint32_t sorted[kWoChunk];         // the chunk's keys in window order: offset | window << 16
  __shared__ uint32_t gdelta[kWoBins];          // window t's perm position minus its local one
  __shared__ uint32_t tsum[2][4];
  __shared__ uint64_t peer_mask[4][kWoBins];    // per wave: the lanes of this step holding each window
  const uint32_t t = threadIdx.x, wave = t >> 6, lane = t & 63u;
  const uint32_t c = xcd_major(blockIdx.x, gridDim.x);
  const uint64_t k0 = (uint64_t)c * kWoChunk;
  const uint32_t kn = (uint32_t)min<uint64_t>(kWoChunk, n - k0);
  // every global load first: the chunk's 4 KiB of window bytes (16 B per thread;
  // the workspace holds whole chunks), window t's total and this chunk's prefix
  const u32x4 cwv = *reinterpret_cast<const u32x4*>(wins + k0 + 16u * t);
  const uint32_t tot = totals[t];
  const uint32_t pre = counts[(uint64_t)c * kWoBins + t] + bsum[(uint64_t)(c / kWoScanBlock) * kWoBins + t];
  cw[4u * t + 0] = cwv.x;
  cw[4u * t + 1] = cwv.y;
  cw[4u * t + 2] = cwv.z;
  cw[4u * t + 3] = cwv.w;
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    next[v][t] = 0;
    peer_mask[v][t] = 0;
  }
  __syncthreads();
  // each wave's histogram of its 1024 window bytes (next[] as counters for now)
  const uint8_t* cwb = reinterpret_cast<const uint8_t*>(cw);
  const uint32_t s0 = kWoSub * wave, s1 = min(kn, s0 + kWoSub);
  uint32_t ws[kWoSub / 64];  // this lane's window in every step
#pragma unroll
  for (uint32_t st = 0; st < kWoSub / 64; ++st) ws[st] = cwb[s0 + 64u * st + lane];
#pragma unroll
  for (uint32_t st = 0; st < kWoSub / 64; ++st)
    if (s0 + 64u * st + lane < s1) atomicAdd(&next[wave][ws[st]], 1u);
  __syncthreads();
  // window t: its keys in the chunk (hc), in waves 0..v-1, and two exclusive scans over
  // the 256 windows: of the totals (the window's base in perm) and of hc (its local start)
  uint32_t hv[4], hc = 0;
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    hv[v] = next[v][t];
    hc += hv[v];
  }
  uint32_t it = tot, ih = hc;
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t ut = (uint32_t)__shfl_up((int)it, d), uh = (uint32_t)__shfl_up((int)ih, d);
    if (lane >= d) {
      it += ut;
      ih += uh;
    }
  }
  if (lane == 63) {
    tsum[0][wave] = it;
    tsum[1][wave] = ih;
  }
  __syncthreads();
  uint32_t bbase = it - tot, lbase = ih - hc;
  for (uint32_t v = 0; v < wave; ++v) {
    bbase += tsum[0][v];
    lbase += tsum[1][v];
  }
  if (c == 0 && win_start) {
    win_start[t] = bbase;
    if (t == kWoThreads - 1) win_start[kWoBins] = bbase + tot;  // = n
  }
  gdelta[t] = bbase + pre - lbase;
  {
    uint32_t run = lbase;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      next[v][t] = run;
      run += hv[v];
    }
  }
  __syncthreads();
  // (1) the chunk's stable window order, in LDS
#pragma unroll
  for (uint32_t st = 0; st < kWoSub / 64; ++st) {
    if (s0 + 64u * st >= s1) break;  // wave-uniform
    const uint32_t i = s0 + 64u * st + lane;
    const uint32_t w = ws[st];
    const bool valid = i < s1;
    if (valid) atomicOr(reinterpret_cast<unsigned long long*>(&peer_mask[wave][w]), 1ull << lane);
    if (valid) {
      const uint64_t peers = peer_mask[wave][w];
      const uint32_t base = next[wave][w];
      const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(peers >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)peers, 0u));
      sorted[base + rank] = i | (w << 16);
      if (rank == 0) {  // one lane per window: no conflict
        next[wave][w] = base + (uint32_t)__popcll(peers);
        peer_mask[wave][w] = 0;
      }
    }
  }
  __syncthreads();
  // (2) out in that order: local position j holds key offset i of window w
  uint32_t e[kWoChunk / kWoThreads];
#pragma unroll
  for (uint32_t q = 0; q < kWoChunk / kWoThreads; ++q) e[q] = sorted[min(t + kWoThreads * q, kn - 1u)];
#pragma unroll
  for (uint32_t q = 0; q < kWoChunk / kWoThreads; ++q) {
    const uint32_t j = t + kWoThreads * q;
    const uint32_t g = gdelta[e[q] >> 16] + j;
    if (j < kn) perm[g] = (uint32_t)(k0 + (e[q] & 0xffffu));
  }
}

}  // namespace

uint64_t win_order_workspace_bytes(uint64_t n) {  // counts, totals, then the window bytes (whole chunks)
  const uint64_t chunks = (n + kWoChunk - 1) / kWoChunk;
  const uint64_t blocks = (chunks + kWoScanBlock - 1) / kWoScanBlock;
  return ((chunks + blocks) * kWoBins + kWoBins) * sizeof(uint32_t) + chunks * kWoChunk;
}

hipError_t launch_win_order(const void* hashes, uint64_t n, uint32_t* perm, uint32_t* win_start, void* workspace,
                            hipStream_t st) {
  if (n == 0) {
    if (win_start) return hipMemsetAsync(win_start, 0, (kWoBins + 1) * sizeof(uint32_t), st);
    return hipSuccess;
  }
  if (n > 0xffffffffull) return hipErrorInvalidValue;  // 32-bit key indices
  const uint32_t chunks = (uint32_t)((n + kWoChunk - 1) / kWoChunk);
  const uint32_t blocks = (chunks + kWoScanBlock - 1) / kWoScanBlock;
  uint32_t* counts = static_cast<uint32_t*>(workspace);
  uint32_t* bsum = counts + (uint64_t)chunks * kWoBins;
  uint32_t* totals = bsum + (uint64_t)blocks * kWoBins;
  uint32_t* wins = totals + kWoBins;  // 16-B aligned: whole rows of 256 u32 before it
  const u32x4* h = static_cast<const u32x4*>(hashes);
  hipLaunchKernelGGL(k_wo_hist, dim3(chunks), dim3(kWoThreads), 0, st, h, n, counts, wins);
  hipLaunchKernelGGL(k_wo_scan_blocks, dim3(blocks), dim3(256), 0, st, counts, chunks, bsum);
  hipLaunchKernelGGL(k_wo_scan_top, dim3(1), dim3(256), 0, st, bsum, blocks, totals);
  hipLaunchKernelGGL(k_wo_scatter, dim3(chunks), dim3(kWoThreads), 0, st, reinterpret_cast<const uint8_t*>(wins), n,
                     chunks, counts, bsum, totals, perm, win_start);
  return hipGetLastError();
}

}  // namespace shfhb
