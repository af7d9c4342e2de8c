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
// Three launches, one workgroup of four waves per chunk of kWoChunk keys:
//   k_wo_hist        (shf_win_order*) the chunk's 256-bin histogram (LDS
//                    atomics) from its 16-B hash records, and each key's window
//                    as one byte; or, when a hashing kernel has written the
//                    window bytes beside its records (shf_hash_batch_*_win*,
//                    kOutHashWin), k_wo_hist_bytes from those bytes (1 B per
//                    key) -- or nothing, when the 16-B hashing kernel counted
//                    the chunks itself (k_fixed16_win);
//   k_wo_scan_rows   the bin-major counts scanned per window, one row each;
//   k_wo_scatter     the chunk ordered in LDS, then written out in order.
// Chunks are dealt to the XCDs in contiguous ranges (workgroup g runs on XCD
// g % 8), so the runs of positions that consecutive chunks write into one
// window's range, and the 128-B lines of the counts rows, fill through one L2.
#include <hip/hip_runtime.h>
#include <stdint.h>

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

// One chunk per workgroup. (1) Each wave walks its 1024 keys in key order, 64
// per step: a lane's rank among the wave's keys of its window = the window's
// count so far (cnt, one plain LDS read) + its rank among the step's peers
// (match_byte: eight ballots); the lowest peer advances the count (one plain
// write; LDS accesses of a wave execute in order, so the next step reads it).
// (2) Per window (thread t = window t): the waves' counts become each wave's
// first local position (exclusive scans over the windows of the chunk counts
// and of the batch totals, and over the waves); gdelta = the window's perm
// position minus its local one (its base from the totals + the chunk's prefix,
// k_wo_scan_rows). (3) Each key's offset goes to sorted[first + rank] (u16).
// (4) The chunk leaves in that order, thread t the positions t, t + 256, ...:
// a window's keys are consecutive both in LDS and in perm, so each store
// instruction writes a few runs of whole lines. Measured against other forms
// per 10M keys (profiles/r4/win_order/README.md): 64-bit LDS peer masks with
// atomic OR and u32 entries (round 3) 26 us; ballots, u32 entries 25; this
// (ballots, u16 entries: 17 KiB of LDS, 7 workgroups per CU) 23; one ordering
// pass after per-wave histograms 24; persistent workgroups prefetching the
// next chunk 28-42; ranks from LDS atomics with return (served in lane order in
// every test, checked) 69.
__global__ __launch_bounds__(kWoThreads) void k_wo_scatter(const uint8_t* __restrict__ wins, uint64_t n,
                                                            const uint32_t* __restrict__ counts,
                                                            uint32_t* __restrict__ perm,
                                                            uint32_t* __restrict__ win_start) {
  __shared__ uint32_t cnt[4][kWoBins];          // per wave: the window's keys so far, then its first position
  __shared__ uint32_t cw[kWoChunk / 4];         // the chunk's window bytes
  __shared__ uint16_t sorted[kWoChunk];         // the chunk's key offsets in window order
  __shared__ uint32_t gdelta[kWoBins];          // window t's perm position minus its local one
  __shared__ uint32_t tsum[2][4];
  const uint32_t t = threadIdx.x, wave = t >> 6, lane = t & 63u;
  const uint32_t c = xcd_major(blockIdx.x, gridDim.x);
  const uint64_t k0 = (uint64_t)c * kWoChunk;
  const uint32_t kn = (uint32_t)min<uint64_t>(kWoChunk, n - k0);
  const uint32_t s0 = kWoSub * wave, s1 = min(kn, s0 + kWoSub);
  const uint32_t* row = counts + (uint64_t)t * wo_row_stride(gridDim.x);
  const uint32_t tot = row[gridDim.x];
  const uint32_t pre = row[c];
  uint32_t ws[kWoSub / 64];  // this lane's window in every step
  {
    const u32x4 cwv = *reinterpret_cast<const u32x4*>(wins + k0 + 16u * t);  // the workspace holds whole chunks
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
    ws[st] = cwb[s0 + 64u * st + lane];
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
    ws[st] = cwb[i];  // read again: not held across the barriers
    if (i < s1) sorted[cnt[wave][ws[st]] + rk[st]] = (uint16_t)i;
  }
  __syncthreads();
#pragma unroll
  for (uint32_t q0 = 0; q0 < kWoChunk / kWoThreads; q0 += 4) {  // four positions at a time (registers)
    uint32_t e[4];
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) {
      const uint32_t j = min(t + kWoThreads * (q0 + q), kn - 1u);
      e[q] = sorted[j];
    }
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) {
      const uint32_t j = t + kWoThreads * (q0 + q);
      const uint32_t w = cwb[e[q]];
      if (j < kn) perm[gdelta[w] + j] = (uint32_t)(k0 + e[q]);
    }
    asm volatile("" ::: "memory");
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
