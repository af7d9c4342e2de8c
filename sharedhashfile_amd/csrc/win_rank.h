// One chunk's stable order by window, computed inside the kernel that has the
// chunk's windows in registers (the 16-B hashing kernel, or the order pass over
// hash records or window bytes), so the order pass after the scan only places
// keys (win_order.hip: k_wo_place). Shared by kernels.hip and win_order.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"

namespace shfhb {

typedef uint32_t wo_u32x4 __attribute__((ext_vector_type(4)));

// The lanes of the wave whose window byte equals this lane's (its "peers",
// itself included): eight ballots, one per bit of the byte, each folded into
// the lanes that differ from this one in that bit (v_bitop3: diff |= m ^ bal).
__device__ __forceinline__ uint64_t wo_match_byte(uint32_t w) {
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

// Wave-wide inclusive scan of a u32 (DPP: shifts by 1, 2, 4, 8 lanes within
// each row of 16, then rows 0 and 1's last lanes added into the rows after
// them): six dependent VALU adds instead of six ds_bpermute round trips.
__device__ __forceinline__ uint32_t wo_wave_incl_scan(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);  // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);  // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);  // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true);  // row_shr:8
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15 into rows 1, 3
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31 into rows 2, 3
  return v;
}

// LDS of one chunk's ranking in a workgroup of WAVES waves.
template <uint32_t WAVES>
struct WoRankLds {
  uint32_t cnt[WAVES][kWoBins];  // per wave: the window's keys so far, then its first position
  __attribute__((aligned(16))) uint16_t sorted[kWoChunk];  // the chunk's key offsets in window order
  uint32_t tsum[4];
};

// Each wave clears its own counts (only it touches them until the barrier
// after the ranking loop, so no barrier is needed before it).
template <uint32_t WAVES>
__device__ __forceinline__ void wo_rank_init(WoRankLds<WAVES>& L) {
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
#pragma unroll
  for (uint32_t e = lane; e < kWoBins; e += 64u) L.cnt[wave][e] = 0;
}

// Key offset in the chunk of wave `wave`'s lane `lane` at step q: each wave
// owns STEPS x 64 consecutive keys, so every load instruction of a wave reads 64
// consecutive records, and waves and steps follow the key order (stability).
template <uint32_t STEPS>
__device__ __forceinline__ uint32_t wo_key_of(uint32_t wave, uint32_t q, uint32_t lane) {
  return (wave * STEPS + q) * 64u + lane;
}

// The chunk's keys [0, kn) with this lane's windows w[q] (key wo_key_of<STEPS>):
// (1) each wave walks its keys in order, 64 per step: a lane's rank among the
// wave's keys of its window = the window's count so far (cnt, one plain LDS
// read) + its rank among the step's peers (wo_match_byte); the lowest peer
// advances the count (one plain write; a wave's LDS accesses execute in order,
// so the next step reads it). (2) Thread b < 256 (window b): the chunk's count
// of window b goes to counts_col[b * stride] (the bin-major counts row), and
// the waves' counts become each wave's first position (exclusive scans over
// the windows and over the waves). (3) Each key's offset goes to
// sorted[first + rank]; (4) the 8-KiB order leaves as 16 B per thread into
// sorted_out[0, 4096) (positions >= kn hold no key). Every thread of the
// workgroup calls it, each wave after its own wo_rank_init(L) (no barrier
// between); a workgroup that reuses L passes a barrier after the last call.
template <uint32_t WAVES, uint32_t STEPS>
__device__ __forceinline__ void wo_rank_chunk(const uint32_t (&w)[STEPS], uint32_t kn, WoRankLds<WAVES>& L,
                                              uint32_t* __restrict__ counts_col, uint64_t stride,
                                              uint16_t* __restrict__ sorted_out) {
  static_assert(WAVES * STEPS * 64u == kWoChunk && WAVES >= 4, "one chunk; at least one thread per window");
  const uint32_t t = threadIdx.x, wave = t >> 6, lane = t & 63u;
  uint32_t rk[STEPS];
#pragma unroll
  for (uint32_t q = 0; q < STEPS; ++q) {
    const bool valid = wo_key_of<STEPS>(wave, q, lane) < kn;
    const uint64_t peers = wo_match_byte(w[q]) & __builtin_amdgcn_ballot_w64(valid);
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(peers >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)peers, 0u));
    const uint32_t base = L.cnt[wave][w[q]];
    rk[q] = base + rank;
    if (valid && rank == 0) L.cnt[wave][w[q]] = base + (uint32_t)__popcll(peers);
  }
  __syncthreads();
  uint32_t hc = 0, ih = 0, hv[WAVES];
  if (t < kWoBins) {
#pragma unroll
    for (uint32_t v = 0; v < WAVES; ++v) {
      hv[v] = L.cnt[v][t];
      hc += hv[v];
    }
    counts_col[(uint64_t)t * stride] = hc;
    ih = wo_wave_incl_scan(hc);
    if (lane == 63) L.tsum[wave] = ih;
  }
  __syncthreads();
  if (t < kWoBins) {
    uint32_t run = ih - hc;
    for (uint32_t v = 0; v < wave; ++v) run += L.tsum[v];
#pragma unroll
    for (uint32_t v = 0; v < WAVES; ++v) {
      L.cnt[v][t] = run;
      run += hv[v];
    }
  }
  __syncthreads();
#pragma unroll
  for (uint32_t q = 0; q < STEPS; ++q) {
    const uint32_t i = wo_key_of<STEPS>(wave, q, lane);
    if (i < kn) L.sorted[L.cnt[wave][w[q]] + rk[q]] = (uint16_t)i;
  }
  __syncthreads();
  for (uint32_t e = t; e < kWoChunk / 8u; e += WAVES * 64u)
    reinterpret_cast<wo_u32x4*>(sorted_out)[e] = reinterpret_cast<const wo_u32x4*>(L.sorted)[e];
}

}  // namespace shfhb
