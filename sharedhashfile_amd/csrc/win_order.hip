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
#include <stdlib.h>

#include <algorithm>

#include "../../include/shf_hash_batch.h"
#include "kernels.h"

namespace shfhb {

namespace {

constexpr uint32_t kWoThreads = 256;                 // 4 waves
constexpr uint32_t kWoSub = kWoChunk / 4;            // keys per wave (16 steps of 64) in the scatter
static_assert(kWoChunk == 4096 && kWoBins == 256, "one chunk = 4 waves x 16 steps x 64 keys; one bin per thread");

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));


__device__ __forceinline__ uint32_t win_of(const u32x4* hashes, uint64_t key) {
  return __builtin_nontemporal_load(&hashes[key]).x & 0xffu;  // h1's low byte (shf.c:800)
}

// One chunk per workgroup: its 256-bin histogram (LDS atomics) as one row of
// counts[c][*] (one coalesced 1-KiB store) and every key's window as one byte.
// Thread t takes keys 256 s + t of step s (each load instruction reads 1 KiB of
// consecutive records); the window bytes gather in LDS and leave as 16 B per
// thread.
__global__ __launch_bounds__(kWoThreads) void k_wo_hist(const u32x4* __restrict__ hashes, uint64_t n,
                                                       uint32_t* __restrict__ counts, uint8_t* __restrict__ wins) {
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
  counts[(uint64_t)t * wo_row_stride(gridDim.x) + c] = hist[t];
  // 16 window bytes per thread (bytes past the batch land in the workspace's last chunk, unused)
  reinterpret_cast<u32x4*>(wins + k0)[t] = reinterpret_cast<const u32x4*>(cwb)[t];
}

// The same histogram from the window bytes a hashing kernel wrote beside its
// records (kOutHashWin): 1 B per key read instead of the 16-B record. Thread t
// takes the chunk's bytes [16 t, 16 t + 16) (one 16-B load; the workspace holds
// whole chunks, bytes past the batch are not counted).
__global__ __launch_bounds__(kWoThreads) void k_wo_hist_bytes(const uint8_t* __restrict__ wins, uint64_t n,
                                                             uint32_t* __restrict__ counts) {
  __shared__ uint32_t hist[kWoBins];
  const uint32_t t = threadIdx.x, c = xcd_major(blockIdx.x, gridDim.x);
  hist[t] = 0;
  const uint64_t k0 = (uint64_t)c * kWoChunk;
  const uint32_t kn = (uint32_t)min<uint64_t>(kWoChunk, n - k0);
  const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(wins + k0) + t);
  __syncthreads();
  const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (uint32_t q = 0; q < 16u; ++q)
    if (16u * t + q < kn) atomicAdd(&hist[(w4[q >> 2] >> (8u * (q & 3u))) & 0xffu], 1u);
  __syncthreads();
  counts[(uint64_t)t * wo_row_stride(gridDim.x) + c] = hist[t];
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
    uint32_t inc = sum;  // inclusive scan of the threads' sums over the wave
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
      const uint32_t u = (uint32_t)__shfl_up((int)inc, d);
      if (lane >= d) inc += u;
    }
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
                                                          const uint32_t* __restrict__ counts,
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
  const uint32_t* row = counts + (uint64_t)t * wo_row_stride(gridDim.x);
  const uint32_t tot = row[gridDim.x];  // window t's keys in the batch (k_wo_scan_rows)
  const uint32_t pre = row[c];          // ... in the chunks before this one
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

// The lanes of the wave whose window byte equals this lane's (its "peers",
// itself included): eight ballots, one per bit of the byte, each folded into
// the lanes that differ from this one in that bit (v_bitop3: diff |= m ^ bal).
__device__ __forceinline__ uint64_t match_byte(uint32_t w) {
  uint32_t lo = 0, hi = 0;
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    // m = 0 or ~0 (this lane's bit b), bal = the lanes whose bit b is set: two VALU ops
    // (written out: the compiler's own sequence for the same ballot takes three)
    uint32_t m;
    uint64_t bal;
    asm volatile("v_bfe_i32 %0, %2, %3, 1\n\tv_cmp_ne_u32_e64 %1, 0, %0" : "=&v"(m), "=s"(bal) : "v"(w), "n"(b));
    lo = __builtin_amdgcn_bitop3_b32(lo, m, (uint32_t)bal, 0xF6);  // lo | (m ^ bal)
    hi = __builtin_amdgcn_bitop3_b32(hi, m, (uint32_t)(bal >> 32), 0xF6);
  }
  return ~(((uint64_t)hi << 32) | lo);
}

// k_wo_scatter with the step's peers found by ballots instead of LDS atomics:
// (1) each wave walks its 1024 keys, 64 per step: a lane's rank among the
// wave's keys of its window = the window's count so far (cnt, read) + its rank
// among the step's peers; the lowest peer advances the count (one plain read and
// one plain write per step, no atomics); (2) per window the waves' counts become
// their first local positions; (3) each key goes to sorted[first + rank];
// (4) out in order, as k_wo_scatter.
__global__ __launch_bounds__(kWoThreads) void k_wo_scatter_ballot(const uint8_t* __restrict__ wins, uint64_t n,
                                                                 const uint32_t* __restrict__ counts,
                                                                 uint32_t* __restrict__ perm,
                                                                 uint32_t* __restrict__ win_start, uint32_t dbg) {
  __shared__ uint32_t cnt[4][kWoBins];   // per wave: the window's keys so far, then its first local position
  __shared__ uint32_t cw[kWoChunk / 4];  // the chunk's window bytes
  __shared__ uint32_t sorted[kWoChunk];  // the chunk's keys in window order: offset | window << 16
  __shared__ uint32_t gdelta[kWoBins];   // window t's perm position minus its local one
  __shared__ uint32_t tsum[2][4];
  const uint32_t t = threadIdx.x, wave = t >> 6, lane = t & 63u;
  const uint32_t c = xcd_major(blockIdx.x, gridDim.x);
  const uint64_t k0 = (uint64_t)c * kWoChunk;
  const uint32_t kn = (uint32_t)min<uint64_t>(kWoChunk, n - k0);
  const uint32_t* row = counts + (uint64_t)t * wo_row_stride(gridDim.x);
  u32x4 cwv = {t * 0x01010101u, 0u, 0u, 0u};
  uint32_t tot = 4096u, pre = c * 16u;
  if (!(dbg & 32)) {
    cwv = *reinterpret_cast<const u32x4*>(wins + k0 + 16u * t);
    tot = row[gridDim.x];
    pre = row[c];
  }
  cw[4u * t + 0] = cwv.x;
  cw[4u * t + 1] = cwv.y;
  cw[4u * t + 2] = cwv.z;
  cw[4u * t + 3] = cwv.w;
#pragma unroll
  for (int v = 0; v < 4; ++v) cnt[v][t] = 0;
  __syncthreads();
  const uint8_t* cwb = reinterpret_cast<const uint8_t*>(cw);
  const uint32_t s0 = kWoSub * wave, s1 = min(kn, s0 + kWoSub);
  uint32_t ws[kWoSub / 64], rk[kWoSub / 64] = {};
#pragma unroll
  for (uint32_t st = 0; st < kWoSub / 64; ++st) ws[st] = cwb[s0 + 64u * st + lane];
  // (1) ranks within the wave
  if (dbg & 1) {
#pragma unroll
    for (uint32_t st = 0; st < kWoSub / 64; ++st) rk[st] = 64u * st + lane;
  } else
#pragma unroll
  for (uint32_t st = 0; st < kWoSub / 64; ++st) {
    const bool valid = s0 + 64u * st + lane < s1;
    const uint64_t peers = ((dbg & 128) ? (1ull << lane) : match_byte(ws[st])) & __builtin_amdgcn_ballot_w64(valid);
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(peers >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)peers, 0u));
    if (dbg & 64) {
      rk[st] = rank + (uint32_t)__popcll(peers);
      continue;
    }
    const uint32_t base = cnt[wave][ws[st]];
    rk[st] = base + rank;
    if (valid && rank == 0) cnt[wave][ws[st]] = base + (uint32_t)__popcll(peers);
  }
  __syncthreads();
  // (2) window t: its keys in the chunk and in waves 0..v-1; exclusive scans over
  // the windows of the totals (its base in perm) and of the chunk counts (its local start)
  uint32_t hv[4], hc = 0;
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    hv[v] = cnt[v][t];
    hc += hv[v];
  }
  uint32_t it = tot, ih = hc;
  if (!(dbg & 16))
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
      cnt[v][t] = (dbg & 1) ? 0u : run;
      run += hv[v];
    }
  }
  __syncthreads();
  // (3) the chunk's stable window order, in LDS
  if (!(dbg & 2))
#pragma unroll
  for (uint32_t st = 0; st < kWoSub / 64; ++st) {
    const uint32_t i = s0 + 64u * st + lane;
    if (i < s1) sorted[(cnt[wave][ws[st]] + rk[st]) & 4095u] = i | (ws[st] << 16);
  }
  __syncthreads();
  // (4) out in that order: local position j holds key offset i of window w
  uint32_t e[kWoChunk / kWoThreads];
#pragma unroll
  for (uint32_t q = 0; q < kWoChunk / kWoThreads; ++q) e[q] = sorted[min(t + kWoThreads * q, kn - 1u)];
#pragma unroll
  for (uint32_t q = 0; q < kWoChunk / kWoThreads; ++q) {
    const uint32_t j = t + kWoThreads * q;
    const uint32_t g = (dbg & 4) ? (uint32_t)k0 + j : min(gdelta[(e[q] >> 16) & 255u] + j, (uint32_t)n - 1u);
    if (j < kn && (!(dbg & 8) || e[q] == 0xffffffffu)) perm[g] = (uint32_t)(k0 + (e[q] & 0xffffu));
  }
}

// k_wo_scatter with each step's ranks taken from LDS atomics that return the
// old count (ds_add_rtn_u32: one instruction per step, no ballots): lanes of a
// step that share a window get consecutive counts, and the stable order needs
// them in lane order. The order is then checked where it is written out (each
// window's run of the sorted chunk must hold increasing key offsets: with the
// counts exact, that is exactly the stable order); a chunk that fails the
// check is ordered again with ballots (k_wo_scatter_ballot's ranks), so the
// result never depends on the order the LDS unit serves same-address lanes in.
__global__ __launch_bounds__(kWoThreads) void k_wo_scatter_fast(const uint8_t* __restrict__ wins, uint64_t n,
                                                               const uint32_t* __restrict__ counts,
                                                               uint32_t* __restrict__ perm,
                                                               uint32_t* __restrict__ win_start, uint32_t dbg) {
  __shared__ uint32_t cnt[4][kWoBins];
  __shared__ uint32_t cw[kWoChunk / 4];
  __shared__ uint32_t sorted[kWoChunk];
  __shared__ uint32_t gdelta[kWoBins];
  __shared__ uint32_t tsum[2][4];
  const uint32_t t = threadIdx.x, wave = t >> 6, lane = t & 63u;
  const uint32_t c = xcd_major(blockIdx.x, gridDim.x);
  const uint64_t k0 = (uint64_t)c * kWoChunk;
  const uint32_t kn = (uint32_t)min<uint64_t>(kWoChunk, n - k0);
  const u32x4 cwv = *reinterpret_cast<const u32x4*>(wins + k0 + 16u * t);
  const uint32_t* row = counts + (uint64_t)t * wo_row_stride(gridDim.x);
  const uint32_t tot = row[gridDim.x];
  const uint32_t pre = row[c];
  cw[4u * t + 0] = cwv.x;
  cw[4u * t + 1] = cwv.y;
  cw[4u * t + 2] = cwv.z;
  cw[4u * t + 3] = cwv.w;
#pragma unroll
  for (int v = 0; v < 4; ++v) cnt[v][t] = 0;
  __syncthreads();
  const uint8_t* cwb = reinterpret_cast<const uint8_t*>(cw);
  const uint32_t s0 = kWoSub * wave, s1 = min(kn, s0 + kWoSub);
  uint32_t ws[kWoSub / 64], rk[kWoSub / 64];
#pragma unroll
  for (uint32_t st = 0; st < kWoSub / 64; ++st) ws[st] = cwb[s0 + 64u * st + lane];
  // (1) ranks within the wave: the window's count so far, one atomic per step
#pragma unroll
  for (uint32_t st = 0; st < kWoSub / 64; ++st)
    rk[st] = s0 + 64u * st + lane < s1 ? atomicAdd(&cnt[wave][ws[st]], 1u) : 0u;
  for (int pass = 0;; ++pass) {
    __syncthreads();
    // (2) window t: its keys in the chunk and in waves 0..v-1; exclusive scans over
    // the windows of the totals (its base in perm) and of the chunk counts (its local start)
    uint32_t hv[4], hc = 0;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      hv[v] = cnt[v][t];
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
    if (c == 0 && win_start && pass == 0) {
      win_start[t] = bbase;
      if (t == kWoThreads - 1) win_start[kWoBins] = bbase + tot;  // = n
    }
    gdelta[t] = bbase + pre - lbase;
    {
      uint32_t run = lbase;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        cnt[v][t] = run;
        run += hv[v];
      }
    }
    __syncthreads();
    // (3) the chunk's window order, in LDS
#pragma unroll
    for (uint32_t st = 0; st < kWoSub / 64; ++st) {
      const uint32_t i = s0 + 64u * st + lane;
      if (i < s1) sorted[cnt[wave][ws[st]] + rk[st]] = i | (ws[st] << 16);
    }
    __syncthreads();
    // the check: within each window's run, key offsets increase
    bool bad = false;
#pragma unroll
    for (uint32_t q = 0; q < kWoChunk / kWoThreads; ++q) {
      const uint32_t j = t + kWoThreads * q;
      if (j != 0 && j < kn) {
        const uint32_t a = sorted[j - 1], b = sorted[j];
        bad |= (a >> 16) == (b >> 16) && (a & 0xffffu) > (b & 0xffffu);
      }
    }
    if (!__syncthreads_or((int)bad) || pass == 1 || (dbg & 1)) break;
    // fallback: ranks from ballots (as k_wo_scatter_ballot), counts rebuilt from zero
#pragma unroll
    for (int v = 0; v < 4; ++v) cnt[v][t] = 0;
    __syncthreads();
#pragma unroll
    for (uint32_t st = 0; st < kWoSub / 64; ++st) {
      const bool valid = s0 + 64u * st + lane < s1;
      const uint64_t peers = match_byte(ws[st]) & __builtin_amdgcn_ballot_w64(valid);
      const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(peers >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)peers, 0u));
      const uint32_t base = cnt[wave][ws[st]];
      rk[st] = base + rank;
      if (valid && rank == 0) cnt[wave][ws[st]] = base + (uint32_t)__popcll(peers);
    }
  }
  // (4) out in that order: local position j holds key offset i of window w
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

// LDS-lean forms of k_wo_scatter_ballot (more workgroups per CU):
//   V = 1: no LDS copy of the window bytes (each lane loads its 16 bytes, one per
//          step, from the workspace), sorted entries u32 (offset | window << 16);
//   V = 2: the window bytes in LDS, sorted entries u16 (the offset; the output
//          pass reads the key's window back from the bytes).
template <int V>
__global__ __launch_bounds__(kWoThreads) void k_wo_scatter_v(const uint8_t* __restrict__ wins, uint64_t n,
                                                            const uint32_t* __restrict__ counts,
                                                            uint32_t* __restrict__ perm,
                                                            uint32_t* __restrict__ win_start) {
  __shared__ uint32_t cnt[4][kWoBins];
  __shared__ uint32_t cw[V == 2 ? kWoChunk / 4 : 1];
  __shared__ uint32_t sorted32[V == 1 ? kWoChunk : 1];
  __shared__ uint16_t sorted16[V == 2 ? kWoChunk : 1];
  __shared__ uint32_t gdelta[kWoBins];
  __shared__ uint32_t tsum[2][4];
  const uint32_t t = threadIdx.x, wave = t >> 6, lane = t & 63u;
  const uint32_t c = xcd_major(blockIdx.x, gridDim.x);
  const uint64_t k0 = (uint64_t)c * kWoChunk;
  const uint32_t kn = (uint32_t)min<uint64_t>(kWoChunk, n - k0);
  const uint32_t s0 = kWoSub * wave, s1 = min(kn, s0 + kWoSub);
  const uint32_t* row = counts + (uint64_t)t * wo_row_stride(gridDim.x);
  const uint32_t tot = row[gridDim.x];
  const uint32_t pre = row[c];
  uint32_t ws[kWoSub / 64];
  if constexpr (V == 1) {
#pragma unroll
    for (uint32_t st = 0; st < kWoSub / 64; ++st) ws[st] = wins[k0 + s0 + 64u * st + lane];
  } else {
    const u32x4 cwv = *reinterpret_cast<const u32x4*>(wins + k0 + 16u * t);
    cw[4u * t + 0] = cwv.x;
    cw[4u * t + 1] = cwv.y;
    cw[4u * t + 2] = cwv.z;
    cw[4u * t + 3] = cwv.w;
  }
#pragma unroll
  for (int v = 0; v < 4; ++v) cnt[v][t] = 0;
  __syncthreads();
  const uint8_t* cwb = reinterpret_cast<const uint8_t*>(cw);
  uint32_t rk[kWoSub / 64];
#pragma unroll
  for (uint32_t st = 0; st < kWoSub / 64; ++st) {
    if constexpr (V == 2) ws[st] = cwb[s0 + 64u * st + lane];
    const bool valid = s0 + 64u * st + lane < s1;
    const uint64_t peers = match_byte(ws[st]) & __builtin_amdgcn_ballot_w64(valid);
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(peers >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)peers, 0u));
    const uint32_t base = cnt[wave][ws[st]];
    rk[st] = base + rank;
    if (valid && rank == 0) cnt[wave][ws[st]] = base + (uint32_t)__popcll(peers);
  }
  __syncthreads();
  uint32_t hv[4], hc = 0;
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    hv[v] = cnt[v][t];
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
      cnt[v][t] = run;
      run += hv[v];
    }
  }
  __syncthreads();
#pragma unroll
  for (uint32_t st = 0; st < kWoSub / 64; ++st) {
    const uint32_t i = s0 + 64u * st + lane;
    if constexpr (V == 2) ws[st] = cwb[i];  // read again: not held across the barriers
    if (i < s1) {
      if constexpr (V == 1) sorted32[cnt[wave][ws[st]] + rk[st]] = i | (ws[st] << 16);
      else sorted16[cnt[wave][ws[st]] + rk[st]] = (uint16_t)i;
    }
  }
  __syncthreads();
#pragma unroll
  for (uint32_t q0 = 0; q0 < kWoChunk / kWoThreads; q0 += 4) {  // four positions at a time (registers)
    uint32_t e[4];
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) {
      const uint32_t j = min(t + kWoThreads * (q0 + q), kn - 1u);
      if constexpr (V == 1) e[q] = sorted32[j];
      else e[q] = sorted16[j];
    }
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) {
      const uint32_t j = t + kWoThreads * (q0 + q);
      const uint32_t w = V == 1 ? (e[q] >> 16) : (uint32_t)cwb[e[q]];
      if (j < kn) perm[gdelta[w] + j] = (uint32_t)(k0 + (e[q] & 0xffffu));
    }
    asm volatile("" ::: "memory");
  }
}

// k_wo_scatter_ballot in one ordering pass: the waves' histograms first (LDS
// adds, no return), so every wave's count per window starts at that window's
// first local position for the wave; each step then places its keys directly
// (base + rank among the step's peers) and the lowest peer advances the count.
// Fewer LDS accesses at random addresses per key (about 4 instead of 5) and no
// ranks held across barriers.
__global__ __launch_bounds__(kWoThreads) void k_wo_scatter_one(const uint8_t* __restrict__ wins, uint64_t n,
                                                              const uint32_t* __restrict__ counts,
                                                              uint32_t* __restrict__ perm,
                                                              uint32_t* __restrict__ win_start) {
  __shared__ uint32_t cnt[4][kWoBins];
  __shared__ uint32_t cw[kWoChunk / 4];
  __shared__ uint32_t sorted[kWoChunk];
  __shared__ uint32_t gdelta[kWoBins];
  __shared__ uint32_t tsum[2][4];
  const uint32_t t = threadIdx.x, wave = t >> 6, lane = t & 63u;
  const uint32_t c = xcd_major(blockIdx.x, gridDim.x);
  const uint64_t k0 = (uint64_t)c * kWoChunk;
  const uint32_t kn = (uint32_t)min<uint64_t>(kWoChunk, n - k0);
  const uint32_t s0 = kWoSub * wave, s1 = min(kn, s0 + kWoSub);
  const uint32_t* row = counts + (uint64_t)t * wo_row_stride(gridDim.x);
  const uint32_t tot = row[gridDim.x];
  const uint32_t pre = row[c];
  const u32x4 cwv = *reinterpret_cast<const u32x4*>(wins + k0 + 16u * t);
  cw[4u * t + 0] = cwv.x;
  cw[4u * t + 1] = cwv.y;
  cw[4u * t + 2] = cwv.z;
  cw[4u * t + 3] = cwv.w;
#pragma unroll
  for (int v = 0; v < 4; ++v) cnt[v][t] = 0;
  __syncthreads();
  const uint8_t* cwb = reinterpret_cast<const uint8_t*>(cw);
  // the wave's histogram of its 1024 window bytes
#pragma unroll
  for (uint32_t st = 0; st < kWoSub / 64; ++st) {
    const uint32_t i = s0 + 64u * st + lane;
    if (i < s1) atomicAdd(&cnt[wave][cwb[i]], 1u);
  }
  __syncthreads();
  uint32_t hv[4], hc = 0;
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    hv[v] = cnt[v][t];
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
      cnt[v][t] = run;
      run += hv[v];
    }
  }
  __syncthreads();
  // each step's keys straight to their local positions
#pragma unroll
  for (uint32_t st = 0; st < kWoSub / 64; ++st) {
    const uint32_t i = s0 + 64u * st + lane;
    const uint32_t w = cwb[i];
    const bool valid = i < s1;
    const uint64_t peers = match_byte(w) & __builtin_amdgcn_ballot_w64(valid);
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(peers >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)peers, 0u));
    const uint32_t base = cnt[wave][w];
    if (valid) sorted[base + rank] = i | (w << 16);
    if (valid && rank == 0) cnt[wave][w] = base + (uint32_t)__popcll(peers);
  }
  __syncthreads();
#pragma unroll
  for (uint32_t q0 = 0; q0 < kWoChunk / kWoThreads; q0 += 8) {
    uint32_t e[8];
#pragma unroll
    for (uint32_t q = 0; q < 8; ++q) e[q] = sorted[min(t + kWoThreads * (q0 + q), kn - 1u)];
#pragma unroll
    for (uint32_t q = 0; q < 8; ++q) {
      const uint32_t j = t + kWoThreads * (q0 + q);
      if (j < kn) perm[gdelta[e[q] >> 16] + j] = (uint32_t)(k0 + (e[q] & 0xffffu));
    }
  }
}

// Persistent variant of k_wo_scatter_ballot: gridDim.x workgroups (a multiple
// of 8), workgroup g on XCD g % 8 walks that XCD's contiguous range of chunks
// with a stride of the XCD's workgroups, and loads the next chunk's window bytes
// and prefixes before ordering the current one (the loads of a chunk are a
// latency the order of the previous one hides). A lane reads its own 16
// window bytes (one per step) straight from the workspace: no LDS copy.
__global__ __launch_bounds__(kWoThreads) void k_wo_scatter_pf(const uint8_t* __restrict__ wins, uint64_t n,
                                                             uint32_t chunks, const uint32_t* __restrict__ counts,
                                                             uint32_t* __restrict__ perm,
                                                             uint32_t* __restrict__ win_start, uint32_t dbg) {
  __shared__ uint32_t cnt[4][kWoBins];
  __shared__ uint32_t sorted[kWoChunk];
  __shared__ uint32_t gdelta[kWoBins];
  __shared__ uint32_t tsum[2][4];
  const uint32_t t = threadIdx.x, wave = t >> 6, lane = t & 63u;
  const uint32_t G = gridDim.x, x = blockIdx.x % 8u, gi = blockIdx.x / 8u, P = G / 8u;
  const uint32_t q = chunks / 8u, r8 = chunks % 8u;
  const uint32_t xc0 = x * q + min(x, r8), xc1 = xc0 + q + (x < r8 ? 1u : 0u);  // this XCD's chunks
  const uint32_t* row = counts + (uint64_t)t * wo_row_stride(chunks);
  const uint32_t tot = row[chunks];
  uint32_t c = xc0 + gi;
  uint32_t nws[kWoSub / 64], npre = 0;
  auto fetch = [&](uint32_t cc) {
    const uint64_t kb = (uint64_t)cc * kWoChunk + kWoSub * wave + lane;
#pragma unroll
    for (uint32_t st = 0; st < kWoSub / 64; ++st) nws[st] = wins[kb + 64u * st];
    npre = row[cc];
  };
  if (c < xc1) fetch(c);
  for (; c < xc1; c += P) {
    uint32_t ws[kWoSub / 64];
#pragma unroll
    for (uint32_t st = 0; st < kWoSub / 64; ++st) ws[st] = nws[st];
    const uint32_t pre = npre;
    if (c + P < xc1) fetch(c + P);
    const uint64_t k0 = (uint64_t)c * kWoChunk;
    const uint32_t kn = (uint32_t)min<uint64_t>(kWoChunk, n - k0);
#pragma unroll
    for (int v = 0; v < 4; ++v) cnt[v][t] = 0;
    __syncthreads();
    const uint32_t s0 = kWoSub * wave, s1 = min(kn, s0 + kWoSub);
    uint32_t rk[kWoSub / 64];
#pragma unroll
    for (uint32_t st = 0; st < kWoSub / 64; ++st) {
      if (dbg & 1) {
        rk[st] = 64u * st + lane;
        continue;
      }
      const bool valid = s0 + 64u * st + lane < s1;
      const uint64_t peers = match_byte(ws[st]) & __builtin_amdgcn_ballot_w64(valid);
      const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(peers >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)peers, 0u));
      const uint32_t base = cnt[wave][ws[st]];
      rk[st] = base + rank;
      if (valid && rank == 0) cnt[wave][ws[st]] = base + (uint32_t)__popcll(peers);
    }
    __syncthreads();
    uint32_t hv[4], hc = 0;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      hv[v] = cnt[v][t];
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
        cnt[v][t] = (dbg & 1) ? 0u : run;
        run += hv[v];
      }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t st = 0; st < kWoSub / 64; ++st) {
      const uint32_t i = s0 + 64u * st + lane;
      if (i < s1) sorted[(dbg & 1) ? i : cnt[wave][ws[st]] + rk[st]] = i | (ws[st] << 16);
    }
    __syncthreads();
    uint32_t e[kWoChunk / kWoThreads];
#pragma unroll
    for (uint32_t qq = 0; qq < kWoChunk / kWoThreads; ++qq) e[qq] = sorted[min(t + kWoThreads * qq, kn - 1u)];
#pragma unroll
    for (uint32_t qq = 0; qq < kWoChunk / kWoThreads; ++qq) {
      const uint32_t j = t + kWoThreads * qq;
      const uint32_t g = (dbg & 4) ? (uint32_t)k0 + j : min(gdelta[(e[qq] >> 16) & 255u] + j, (uint32_t)n - 1u);
      if (j < kn) perm[g] = (uint32_t)(k0 + (e[qq] & 0xffffu));
    }
    // the next chunk's first LDS writes (cnt) follow every wave's reads of this one's
    __syncthreads();
  }
}

}  // namespace

// Workspace: the counts (bin-major rows, wo_row_stride), then the window bytes
// (whole chunks; 16-B aligned: the rows are whole multiples of 256 B).
uint64_t win_order_workspace_bytes(uint64_t n) {
  const uint64_t chunks = (n + kWoChunk - 1) / kWoChunk;
  return kWoBins * wo_row_stride(chunks) * sizeof(uint32_t) + chunks * kWoChunk;
}

uint32_t* win_order_counts(void* workspace) { return static_cast<uint32_t*>(workspace); }

uint8_t* win_order_wins(void* workspace, uint64_t n) {
  const uint64_t chunks = (n + kWoChunk - 1) / kWoChunk;
  return reinterpret_cast<uint8_t*>(win_order_counts(workspace) + kWoBins * wo_row_stride(chunks));
}

// The scan and the scatter over counts and window bytes already in the
// workspace (hist_done), or after counting the window bytes.
hipError_t launch_win_order_bytes(uint64_t n, bool hist_done, uint32_t* perm, uint32_t* win_start, void* workspace,
                                  hipStream_t st) {
  if (n == 0) {
    if (win_start) return hipMemsetAsync(win_start, 0, (kWoBins + 1) * sizeof(uint32_t), st);
    return hipSuccess;
  }
  if (n > 0xffffffffull) return hipErrorInvalidValue;  // 32-bit key indices
  const uint32_t chunks = (uint32_t)((n + kWoChunk - 1) / kWoChunk);
  uint32_t* counts = win_order_counts(workspace);
  const uint8_t* wins = win_order_wins(workspace, n);
  if (!hist_done) hipLaunchKernelGGL(k_wo_hist_bytes, dim3(chunks), dim3(kWoThreads), 0, st, wins, n, counts);
  hipLaunchKernelGGL(k_wo_scan_rows, dim3(kWoBins), dim3(256), 0, st, counts, chunks);
  const char* e = getenv("SHF_HB_WO_SCATTER");  // EXPERIMENT (removed once a variant is chosen)
  if (e && e[0] == '2')
    hipLaunchKernelGGL(k_wo_scatter_ballot, dim3(chunks), dim3(kWoThreads), 0, st, wins, n, counts, perm, win_start,
                       (uint32_t)atoi(e + 1));
  else if (e && e[0] == '5' && e[1] == '1')
    hipLaunchKernelGGL(k_wo_scatter_v<1>, dim3(chunks), dim3(kWoThreads), 0, st, wins, n, counts, perm, win_start);
  else if (e && e[0] == '5' && e[1] == '2')
    hipLaunchKernelGGL(k_wo_scatter_v<2>, dim3(chunks), dim3(kWoThreads), 0, st, wins, n, counts, perm, win_start);
  else if (e && e[0] == '6')
    hipLaunchKernelGGL(k_wo_scatter_one, dim3(chunks), dim3(kWoThreads), 0, st, wins, n, counts, perm, win_start);
  else if (e && e[0] == '4')
    hipLaunchKernelGGL(k_wo_scatter_fast, dim3(chunks), dim3(kWoThreads), 0, st, wins, n, counts, perm, win_start,
                       (uint32_t)atoi(e + 1));
  else if (e && e[0] == '3') {  // 3<wgs per CU><dbg>
    const uint32_t per_cu = (uint32_t)(e[1] - '0');
    const uint32_t g = std::min<uint32_t>((chunks + 7u) / 8u * 8u, 256u * per_cu);
    hipLaunchKernelGGL(k_wo_scatter_pf, dim3(g), dim3(kWoThreads), 0, st, wins, n, chunks, counts, perm, win_start,
                       (uint32_t)atoi(e + 2));
  }
  else
    hipLaunchKernelGGL(k_wo_scatter, dim3(chunks), dim3(kWoThreads), 0, st, wins, n, counts, perm, win_start);
  return hipGetLastError();
}

hipError_t launch_win_order(const void* hashes, uint64_t n, uint32_t* perm, uint32_t* win_start, void* workspace,
                            hipStream_t st) {
  if (n == 0 || n > 0xffffffffull) return launch_win_order_bytes(n, true, perm, win_start, workspace, st);
  const uint32_t chunks = (uint32_t)((n + kWoChunk - 1) / kWoChunk);
  hipLaunchKernelGGL(k_wo_hist, dim3(chunks), dim3(kWoThreads), 0, st, static_cast<const u32x4*>(hashes), n,
                     win_order_counts(workspace), win_order_wins(workspace, n));
  return launch_win_order_bytes(n, true, perm, win_start, workspace, st);
}

}  // namespace shfhb
