// Batch key-hashing kernels for MI355X (gfx950).
//
// Each kernel computes, for every key of a batch, exactly what the reference's
// shf_make_hash() leaves in the thread-local SHF_HASH
// (/root/reference/src/shf.c:450-462 -> murmurhash3.c:75-160), or the packed
// UID parts that put/find derive from it (shf.c:800-803, :893-896), or that
// hash's row pre-probe against a device copy of the store's rows (the row scan
// of shf.c:886-922).
//
// Kernels (see DESIGN.md for the roofline of each):
//   k_fixed16   key_len == 16: one lane per key, one 16-B coalesced load and one
//               16-B coalesced store per lane. HBM-bound (32 B/key).
//   k_tiled     key_len % 16 == 0, key_len >= 32 (the 256-B config): a wave owns
//               64 keys; every round it stages 8 or 16 pieces of 16 B of each key
//               through LDS with fully-used segment loads, XOR-swizzled so the
//               lane-per-key ds_read_b128 reads are bank-conflict free.
//   k_span      variable-length keys and most other fixed lengths: a wave owns a
//               tile of 64 consecutive keys = one contiguous span, fetched with
//               1-KiB raw buffer loads, staged in LDS, hashed lane-per-key.
//   k_vround    variable-length keys streamed 128 B per key per round through
//               144-B LDS windows (short / very long keys, k_span's overflow).
//   k_generic   any length, fixed or variable (offset array): one lane per key,
//               64-B per-lane bursts of dword-aligned loads, funnel-shifted with
//               v_alignbyte_b32 for unaligned key starts.
//   k_probe_hashes  row pre-probe of precomputed hashes.
// Every hashing kernel takes its output as a Sink (kernels.h): 16-B hashes,
// 8-B UID parts, or 16-B probe records (+ optional hashes).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <stdlib.h>

#include <algorithm>

#include "murmur3_mix.h"
#include "kernels.h"
#include "win_rank.h"

namespace shfhb {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) const u32x4 g_u32x4;          // global-memory views
typedef __attribute__((address_space(1))) const u32x4_a4 g_u32x4_a4;
typedef __attribute__((address_space(1))) const uint32_t g_u32;

// ---------------------------------------------------------------------------
// Row pre-probe: the row scan of shf_find_key_internal()
// (/root/reference/src/shf.c:886-922) against a device copy of the store's rows.
//   win/tab2/row/rnd from the hash      shf.c:893-896
//   tab = wins[win].tabs[tab2].tab      shf.c:906   (folded into tab_slot)
//   candidate ref: pos != 0, rnd == rnd, tab == tab2, first in ref order  shf.c:919-922
// SHF_REF_MMAP (shf.private.h:48-52) is {u32 tab:11 | rnd:21 << 11, u32 pos}, so
// a ref matches when its first word equals tab2 | rnd << 11 and pos != 0.
// Record (shf_probe, shf_hash_batch.h): {uid, pos, mask | tab << 16, slot}.
// ---------------------------------------------------------------------------
constexpr uint32_t kProbeNone = 0xffffffffu;  // SHF_UID_NONE (shf.h:354) / no slot
constexpr uint32_t kRowsPerTabShift = 16;     // 512 rows x 128 B = 64 KiB per slot

// Two steps, so that the row loads of several keys can be in flight together:
// probe_locate (the 4-B tab_slot lookup) and probe_scan (the row's 8 x 16-B
// loads and 16 compares). The row loads are unconditional: a key whose tab is
// not indexed scans a stand-in (the first 128 B of the tab map, always mapped)
// and its result is discarded.
struct ProbeLoc {
  uint32_t win, tab2, row, want, e;
};

// The map entry comes from the compact map when the index has one (512 KiB of
// ranks + the windows' distinct entries, which stay in L2 beside the row stream
// where the 2-MiB tab_slot map did not: +20 % at 10M keys, profiles/r3/ab_mapsize.txt).
__device__ __forceinline__ ProbeLoc probe_locate(const Sink& k, const State& s) {
  ProbeLoc p;
  const uint32_t lo = (uint32_t)s.h1;
  p.win = lo & 0xffu;
  p.tab2 = (lo >> 16) & 0x7ffu;
  p.row = (uint32_t)(s.h1 >> 32) & 0x1ffu;
  p.want = p.tab2 | (((uint32_t)s.h2 & 0x1fffffu) << 11);
  const uint32_t at = (p.win << 11) | p.tab2;
  if (k.map8) {
    const uint32_t r = reinterpret_cast<const __attribute__((address_space(1))) uint8_t*>(
        reinterpret_cast<uintptr_t>(k.map8))[at];
    if (r < kMapRanks) p.e = reinterpret_cast<g_u32*>(reinterpret_cast<uintptr_t>(k.win_tab))[(p.win << 8) | r];
    else if (r == kMapNone) p.e = kProbeNone;
    else p.e = reinterpret_cast<g_u32*>(reinterpret_cast<uintptr_t>(k.tab_slot))[at];
  } else {
    p.e = reinterpret_cast<g_u32*>(reinterpret_cast<uintptr_t>(k.tab_slot))[at];
  }
  return p;
}

__device__ __forceinline__ bool probe_indexed(const Sink& k, const ProbeLoc& p) {
  return p.e != kProbeNone && (uint64_t)(p.e >> 11) < k.n_slots;
}

// The key's row, or the stand-in when its tab is not indexed.
__device__ __forceinline__ uintptr_t probe_row_addr(const Sink& k, const ProbeLoc& p) {
  return probe_indexed(k, p) ? reinterpret_cast<uintptr_t>(k.rows) + ((uint64_t)(p.e >> 11) << kRowsPerTabShift) +
                                   (p.row << 7)
                             : reinterpret_cast<uintptr_t>(k.tab_slot);
}

// The 16 compares of a row already in registers, and the record.
__device__ __forceinline__ u32x4 probe_match(const Sink& k, const ProbeLoc& p, const u32x4 (&v)[8]) {
  const uint32_t slot = p.e >> 11;
  const bool indexed = probe_indexed(k, p);
  uint32_t mask = 0, pos = 0, first = 0;
#pragma unroll
  for (int q = 7; q >= 0; --q) {  // descending: the lowest matching ref is written last
    if (v[q].w != 0u && v[q].z == p.want) {
      mask |= 2u << (2 * q);
      pos = v[q].w;
      first = 2 * q + 1;
    }
    if (v[q].y != 0u && v[q].x == p.want) {
      mask |= 1u << (2 * q);
      pos = v[q].y;
      first = 2 * q;
    }
  }
  u32x4 rec = {kProbeNone, 0u, 0xffffu << 16, kProbeNone};
  if (indexed) {
    rec.x = mask ? (p.win | (p.tab2 << 8) | (p.row << 19) | (first << 28)) : kProbeNone;
    rec.y = pos;
    rec.z = mask | ((p.e & 0x7ffu) << 16);
    rec.w = slot;
  }
  return rec;
}

__device__ __forceinline__ u32x4 probe_scan(const Sink& k, const ProbeLoc& p) {
  const g_u32x4* r = reinterpret_cast<const g_u32x4*>(probe_row_addr(k, p));
  u32x4 v[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) v[q] = r[q];
  return probe_match(k, p, v);
}

__device__ __forceinline__ u32x4 probe_row(const Sink& k, const State& s) { return probe_scan(k, probe_locate(k, s)); }

// probe_scan for a whole wave (every lane must call it): the rows are fetched
// 8 lanes per row, so each of the 8 load instructions touches 8 whole 128-B
// lines instead of 64 partial ones (row addresses move by __shfl), then
// transposed through `lds` (8 KiB for this wave, XOR-swizzled so both the
// ds_write_b128 and the ds_read_b128 are conflict-free) for the lane's compares:
// +3 % over per-lane row loads (profiles/r1/ab_probe_lds/).
__device__ __forceinline__ u32x4 probe_scan_coop(const Sink& k, const ProbeLoc& p, u32x4* lds) {
  const uint32_t lane = __lane_id();
  const uint64_t at = probe_row_addr(k, p);
  const int alo = (int)(uint32_t)at, ahi = (int)(uint32_t)(at >> 32);
  u32x4 g[8];
#pragma unroll
  for (uint32_t q = 0; q < 8; ++q) {
    const int src = (int)(8u * q + (lane >> 3));
    const uint64_t a = (uint64_t)(uint32_t)__shfl(alo, src) | ((uint64_t)(uint32_t)__shfl(ahi, src) << 32);
    g[q] = *reinterpret_cast<const g_u32x4*>(a + 16u * (lane & 7u));
  }
#pragma unroll
  for (uint32_t q = 0; q < 8; ++q) {
    const uint32_t src = 8u * q + (lane >> 3);
    lds[src * 8u + ((lane & 7u) ^ (src & 7u))] = g[q];
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  u32x4 v[8];
#pragma unroll
  for (uint32_t q = 0; q < 8; ++q) v[q] = lds[lane * 8u + (q ^ (lane & 7u))];
  return probe_match(k, p, v);
}

// Results are stored nontemporally: they are never read back by the kernel, and
// streaming them past the caches measured +3.2 % on 100M x 16-B keys, +6.7 % on
// 256-B keys and +5.4 % on U[8,512] B keys (profiles/r3/ab_ntstore.txt; only a
// batch re-hashed while it still sits in the Infinity Cache loses, -4 %).
__device__ __forceinline__ void store_probe(const Sink& sink, uint64_t i, const State& s, const u32x4& rec) {
  if (sink.hash_out) {
    const u32x4 v = {(uint32_t)s.h1, (uint32_t)(s.h1 >> 32), (uint32_t)s.h2, (uint32_t)(s.h2 >> 32)};
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(sink.hash_out) + i);
  }
  __builtin_nontemporal_store(rec, reinterpret_cast<u32x4*>(sink.out) + i);
}

template <int OUT>
__device__ __forceinline__ void store_result(const Sink& sink, uint64_t i, const State& s) {
  if constexpr (OUT == kOutHash || OUT == kOutHashWin) {
    const u32x4 v = {(uint32_t)s.h1, (uint32_t)(s.h1 >> 32), (uint32_t)s.h2, (uint32_t)(s.h2 >> 32)};
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(sink.out) + i);
    if constexpr (OUT == kOutHashWin) sink.wins[i] = (uint8_t)s.h1;  // the window, shf.c:800
  } else if constexpr (OUT == kOutUid || OUT == kOutUidWin) {
    __builtin_nontemporal_store(uid_parts(s), reinterpret_cast<uint64_t*>(sink.out) + i);
    if constexpr (OUT == kOutUidWin) sink.wins[i] = (uint8_t)s.h1;  // the window, shf.c:800
  } else {
    store_probe(sink, i, s, probe_row(sink, s));
  }
}

// Probe precomputed hashes: one lane per key.
// (A wave-cooperative variant -- 8 lanes per row, matches gathered with
// ballots and ds_bpermute -- measured 3.9x slower: profiles/r1/ab_probe_coop_vs_lane_*.txt.)
__global__ __launch_bounds__(256) void k_probe_hashes(const u32x4* __restrict__ hashes, uint64_t n, Sink sink) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  __shared__ u32x4 rows_lds[256 * 8];
  u32x4 h = {0u, 0u, 0u, 0u};  // lanes past n still take part in the wave's row fetch
  if (i < n) h = __builtin_nontemporal_load(&hashes[i]);
  const State s{pack64(h.x, h.y), pack64(h.z, h.w)};
  const u32x4 rec = probe_scan_coop(sink, probe_locate(sink, s), rows_lds + (threadIdx.x & ~63u) * 8u);
  if (i < n) reinterpret_cast<u32x4*>(sink.out)[i] = rec;
}

// ---------------------------------------------------------------------------
// Variable-length key check (include/shf_hash_batch.h: every key length must be
// < 2^31, the reference's `const int len`, murmurhash3.c:75). A key whose
// offsets decrease or span 2^31 bytes or more is skipped -- its bytes are never
// read, its record never written -- and the call's status word is set.
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool var_key_bad(uint64_t o0, uint64_t o1) { return o1 < o0 || o1 - o0 > 0x7fffffffull; }

__device__ __forceinline__ void flag_bad_key(const Sink& sink) {
  if (sink.status) *reinterpret_cast<volatile uint32_t*>(sink.status) = 1u;
}

// ---------------------------------------------------------------------------
// key_len == 16
// ---------------------------------------------------------------------------
// One key per lane and as many workgroups as keys need: no grid-stride loop
// (6.36 vs 5.16 TB/s at 100M keys against a 8192-block grid-stride loop,
// profiles/r1/ab_fixed16.txt; a loop that runs once measured the same,
// profiles/r1/ab_fixed16_noloop_*.txt). 128/512/1024 threads per block, two keys
// per lane and nontemporal stores all measured within 3 % of this shape
// (profiles/r1/ab_fixed16_shapes/); two or four keys per lane in the fused
// probe ~2 % slower. OUT = kOutProbe is the fused hash + row pre-probe.
constexpr uint32_t kF16Block = 256;

template <int OUT>
__global__ __launch_bounds__(kF16Block) void k_fixed16(const u32x4* __restrict__ keys, uint64_t n, uint32_t seed,
                                                       Sink sink) {
  const uint64_t i = (uint64_t)blockIdx.x * kF16Block + threadIdx.x;
  if constexpr (OUT == kOutProbe) {
    // every lane of the wave takes part in the cooperative row fetch
    const u32x4 k = i < n ? __builtin_nontemporal_load(&keys[i]) : u32x4{0u, 0u, 0u, 0u};
    State s{seed, seed};
    body_block(s, pack64(k.x, k.y), pack64(k.z, k.w));
    finish(s, 16);
    __shared__ u32x4 rows_lds[kF16Block * 8];
    const u32x4 rec = probe_scan_coop(sink, probe_locate(sink, s), rows_lds + (threadIdx.x & ~63u) * 8u);
    if (i < n) store_probe(sink, i, s, rec);
    return;
  }
  if (i >= n) return;
  const u32x4 k = __builtin_nontemporal_load(&keys[i]);
  State s{seed, seed};
  body_block(s, pack64(k.x, k.y), pack64(k.z, k.w));
  finish(s, 16);
  store_result<OUT>(sink, i, s);
}

// 16-B keys hashed and ranked for the window order in one pass (kOutHashWin):
// one workgroup per kWoChunk-key chunk, kWoChunk / BLOCK keys per lane (wave v
// owns keys [v * 64 kKpl, (v + 1) * 64 kKpl), 64 consecutive records per load
// instruction; all of a lane's loads in flight before the first key is hashed).
// Beside each hash record it ranks the chunk by window (win_rank.h: ballots,
// per-wave counts and scans in LDS -- VALU and LDS work this HBM-bound kernel
// has room for) and writes the chunk's 256 window counts and its order (4096
// u16 offsets): the order passes then never read the 16-B records back, and the
// placement after the scan is one load and one store per key (win_order.hip).
constexpr uint32_t kF16WinBlock = 1024;

template <uint32_t BLOCK>
__global__ __launch_bounds__(BLOCK) void k_fixed16_win(const u32x4* __restrict__ keys, uint64_t n, uint32_t seed,
                                                       Sink sink) {
  constexpr uint32_t kKpl = kWoChunk / BLOCK, kWaves = BLOCK / 64u;
  __shared__ WoRankLds<kWaves> L;
  const uint32_t t = threadIdx.x, wave = t >> 6, lane = t & 63u;
  const uint32_t c = xcd_major(blockIdx.x, gridDim.x);
  const uint64_t k0 = (uint64_t)c * kWoChunk;
  const uint32_t kn = (uint32_t)min<uint64_t>(kWoChunk, n - k0);
  wo_rank_init(L);
  u32x4 k[kKpl];  // past the batch: the last key again (hashed, neither stored nor ranked)
#pragma unroll
  for (uint32_t j = 0; j < kKpl; ++j)
    k[j] = __builtin_nontemporal_load(&keys[k0 + min(wo_key_of<kKpl>(wave, j, lane), kn - 1u)]);
  uint32_t w[kKpl];
#pragma unroll
  for (uint32_t j = 0; j < kKpl; ++j) {
    const uint32_t i = wo_key_of<kKpl>(wave, j, lane);
    State s{seed, seed};
    body_block(s, pack64(k[j].x, k[j].y), pack64(k[j].z, k[j].w));
    finish(s, 16);
    w[j] = (uint32_t)s.h1 & 0xffu;  // the window, shf.c:800
    if (i < kn) {
      const u32x4 v = {(uint32_t)s.h1, (uint32_t)(s.h1 >> 32), (uint32_t)s.h2, (uint32_t)(s.h2 >> 32)};
      __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(sink.out) + k0 + i);
    }
  }
  wo_rank_chunk<kWaves, kKpl>(w, kn, L, sink.win_counts + c, wo_row_stride(gridDim.x), sink.win_sorted + k0);
}

// ---------------------------------------------------------------------------
// Generic: one lane per key, any alignment, any length.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t low_bytes_mask(uint32_t nbytes) {
  return nbytes >= 8 ? ~0ull : ((1ull << (8 * nbytes)) - 1ull);
}

// Hash `len` bytes at `p` (any alignment). Only dwords that hold at least one
// byte of the key are ever loaded, so no access can cross into an unmapped page.
__device__ __forceinline__ State hash_bytes(const uint8_t* p, uint32_t len, uint32_t seed) {
  const uintptr_t addr = reinterpret_cast<uintptr_t>(p);
  const uint32_t sh = (uint32_t)(addr & 3u);
  const g_u32* w = reinterpret_cast<const g_u32*>(addr - sh);
  const uint32_t nblocks = len >> 4;
  State s{seed, seed};

  uint32_t j = 0;
  for (; j + 4 <= nblocks; j += 4) {  // 64-B burst per lane
    const g_u32x4_a4* v = reinterpret_cast<const g_u32x4_a4*>(w + 4 * j);
    const u32x4 a = v[0], b = v[1], c = v[2], d = v[3];
    const uint32_t e = sh ? w[4 * j + 16] : 0u;
    const uint32_t x[17] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w, d.x, d.y, d.z, d.w, e};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t d0 = __builtin_amdgcn_alignbyte(x[4 * q + 1], x[4 * q + 0], sh);
      const uint32_t d1 = __builtin_amdgcn_alignbyte(x[4 * q + 2], x[4 * q + 1], sh);
      const uint32_t d2 = __builtin_amdgcn_alignbyte(x[4 * q + 3], x[4 * q + 2], sh);
      const uint32_t d3 = __builtin_amdgcn_alignbyte(x[4 * q + 4], x[4 * q + 3], sh);
      body_block(s, pack64(d0, d1), pack64(d2, d3));
    }
  }
  for (; j < nblocks; ++j) {
    const u32x4 a = *reinterpret_cast<const g_u32x4_a4*>(w + 4 * j);
    const uint32_t e = sh ? w[4 * j + 4] : 0u;
    const uint32_t d0 = __builtin_amdgcn_alignbyte(a.y, a.x, sh);
    const uint32_t d1 = __builtin_amdgcn_alignbyte(a.z, a.y, sh);
    const uint32_t d2 = __builtin_amdgcn_alignbyte(a.w, a.z, sh);
    const uint32_t d3 = __builtin_amdgcn_alignbyte(e, a.w, sh);
    body_block(s, pack64(d0, d1), pack64(d2, d3));
  }

  const uint32_t rem = len & 15u;
  if (rem) {
    const g_u32* t = w + 4 * nblocks;
    const uint32_t need = sh + rem;  // bytes spanned from the aligned base
    uint32_t x[5];
#pragma unroll
    for (int q = 0; q < 5; ++q) x[q] = (4u * q < need) ? t[q] : 0u;
    const uint32_t d0 = __builtin_amdgcn_alignbyte(x[1], x[0], sh);
    const uint32_t d1 = __builtin_amdgcn_alignbyte(x[2], x[1], sh);
    const uint32_t d2 = __builtin_amdgcn_alignbyte(x[3], x[2], sh);
    const uint32_t d3 = __builtin_amdgcn_alignbyte(x[4], x[3], sh);
    const uint64_t t1 = pack64(d0, d1) & low_bytes_mask(rem);
    const uint64_t t2 = rem > 8 ? (pack64(d2, d3) & low_bytes_mask(rem - 8)) : 0ull;
    tail_block(s, t1, t2, rem);
  }
  finish(s, len);
  return s;
}

constexpr unsigned kGenericGridCap = 1u << 20;  // one key per lane: 5.57 vs 5.19 TB/s at 32-B keys
template <int OUT, bool VAR>
__global__ __launch_bounds__(256) void k_generic(const uint8_t* __restrict__ bytes,
                                                 const uint64_t* __restrict__ offsets, uint64_t off_base,
                                                 uint32_t key_len, uint64_t n, uint32_t seed,
                                                 Sink sink) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    uint64_t start;
    uint32_t len;
    if constexpr (VAR) {
      const uint64_t o0 = offsets[i], o1 = offsets[i + 1];
      if (var_key_bad(o0, o1)) {
        flag_bad_key(sink);
        continue;
      }
      start = o0 - off_base;
      len = (uint32_t)(o1 - o0);
    } else {
      start = i * (uint64_t)key_len;
      len = key_len;
    }
    const State s = hash_bytes(bytes + start, len, seed);
    store_result<OUT>(sink, i, s);
  }
}

// ---------------------------------------------------------------------------
// Tiled: key_len % 16 == 0 and key_len >= 32. One wave = 64 keys; each round
// moves 8 blocks (128 B) of every key through an 8-KiB LDS tile per wave.
//
// Load mapping (round r, instruction q = 0..7): lane l fetches 16 B of key
// 8q + l/8 at byte 128r + 16(l%8): 8 lanes read one contiguous 128-B segment.
// LDS layout: key k's piece j sits at k*128 + 16*(j ^ ((k >> 1) & 7)). Writes
// (8 lanes per row) cover a row's 32 banks once; the lane-per-key reads of one
// piece index hit 16 distinct (k&1, slot) pairs per ds_read_b128 lane group, so
// both sides are conflict free.
// The grid is sized to exactly the resident workgroups (launch_fixed), every
// wave walks tiles with a grid stride and prefetches round r+1 into registers
// while hashing round r out of LDS.
// ---------------------------------------------------------------------------
constexpr int kTileKeys = 64;
// One wave per workgroup (4 % faster than 4 at 100M x 256 B) and one tile per
// wave: a grid of as many workgroups as tiles (6.09 vs 5.05 TB/s for a
// persistent grid of the resident workgroups, profiles/r1/ab_tiled_grid.txt).
constexpr int kTiledWaves = 1;  // waves per workgroup
constexpr int kTiledBatchMax = 8;  // LDS blocks read at once (all 8 beat smaller batches: 5.43 vs 4.94 TB/s)

// LDS slot of piece j of key k for R pieces (16 B each) per key per round. The
// XOR term spreads the 16 lanes of each ds_read_b128 lane group (which always
// hold 16 distinct values of k & 15) over 16 distinct 16-B bank slots.
template <int R>
__device__ __forceinline__ uint32_t tile_slot(uint32_t key, uint32_t piece) {
  constexpr uint32_t rows_per_bank_row = 16 / R;  // R=4: 4, R=8: 2, R=16: 1
  return key * (R * 16) + 16u * (piece ^ ((key / rows_per_bank_row) & (R - 1)));
}

template <int OUT, int R>
__global__ __launch_bounds__(64 * kTiledWaves) void k_tiled(const uint8_t* __restrict__ keys, uint32_t key_len,
                                                            uint64_t n, uint32_t seed, Sink sink) {
  static_assert(R == 4 || R == 8 || R == 16, "pieces per key per round");
  constexpr int kTiledBatch = kTiledBatchMax < R ? kTiledBatchMax : R;
  constexpr uint32_t kKeysPerInstr = 64 / R;
  __shared__ __attribute__((aligned(16))) uint8_t lds[kTiledWaves][kTileKeys * R * 16];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = threadIdx.x >> 6;
  uint8_t* tile = lds[wave];

  const uint32_t nblocks = key_len >> 4;
  const uint32_t rounds = (nblocks + R - 1) / R;
  const uint64_t ntiles = (n + kTileKeys - 1) / kTileKeys;
  const uint64_t wstride = (uint64_t)gridDim.x * kTiledWaves;
  uint64_t t = (uint64_t)blockIdx.x * kTiledWaves + wave;
  if (t >= ntiles) return;

  const uint32_t ld_key_sub = lane / R;  // + kKeysPerInstr * q
  const uint32_t ld_piece = lane % R;

  // Fetch round r of tile t into registers (R x 16 B per lane): instruction q
  // reads kKeysPerInstr keys, R lanes per key covering 16R contiguous bytes.
  auto fetch = [&](uint64_t tt, uint32_t r, u32x4 (&reg)[R]) {
    const uint64_t k0 = tt * kTileKeys;
    const uint32_t rb = min((uint32_t)R, nblocks - r * R);
    const bool full = rb == (uint32_t)R && k0 + kTileKeys <= n;
    const uint8_t* src0 = keys + (k0 + ld_key_sub) * key_len + (uint64_t)r * (16u * R) + 16u * ld_piece;
    if (full) {  // common case: no per-lane predicate
#pragma unroll
      for (int q = 0; q < R; ++q)
        reg[q] = __builtin_nontemporal_load(
            reinterpret_cast<const u32x4*>(src0 + (uint64_t)(kKeysPerInstr * q) * key_len));
    } else {
#pragma unroll
      for (int q = 0; q < R; ++q) {
        const uint64_t key = k0 + kKeysPerInstr * q + ld_key_sub;
        reg[q] = (key < n && ld_piece < rb) ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(
                                                  src0 + (uint64_t)(kKeysPerInstr * q) * key_len))
                                            : u32x4{0u, 0u, 0u, 0u};
      }
    }
  };

  u32x4 nxt[R];
  fetch(t, 0, nxt);
  uint32_t r = 0;
  State s{seed, seed};
  while (true) {
    // Stage the fetched round into LDS.
#pragma unroll
    for (int q = 0; q < R; ++q)
      *reinterpret_cast<u32x4*>(tile + tile_slot<R>(kKeysPerInstr * q + ld_key_sub, ld_piece)) = nxt[q];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    const uint32_t rb = min((uint32_t)R, nblocks - r * R);
    // Read this round's blocks of this lane's key, kTiledBatch at a time (all of
    // a batch in flight at once; smaller batches trade ILP for VGPRs/occupancy).
    u32x4 b[kTiledBatch];
    auto read_batch = [&](int j0) {
#pragma unroll
      for (int j = 0; j < kTiledBatch; ++j)
        b[j] = ((uint32_t)(j0 + j) < rb)
                   ? *reinterpret_cast<const u32x4*>(tile + tile_slot<R>(lane, (uint32_t)(j0 + j)))
                   : u32x4{0u, 0u, 0u, 0u};
    };
    read_batch(0);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    // Prefetch the next round (or the next tile's first round).
    uint64_t t_next = t;
    uint32_t r_next = r + 1;
    if (r_next == rounds) {
      t_next = t + wstride;
      r_next = 0;
    }
    const bool more = t_next < ntiles;
    if (more) fetch(t_next, r_next, nxt);

#pragma unroll
    for (int j0 = 0; j0 < R; j0 += kTiledBatch) {
      if (j0) read_batch(j0);
#pragma unroll
      for (int j = 0; j < kTiledBatch; ++j)
        if ((uint32_t)(j0 + j) < rb) body_block(s, pack64(b[j].x, b[j].y), pack64(b[j].z, b[j].w));
    }
    // every lane's reads of this round precede the next round's staging writes
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    if (r + 1 == rounds) {
      const uint64_t key = t * kTileKeys + lane;
      finish(s, key_len);
      if (key < n) store_result<OUT>(sink, key, s);
      s = State{seed, seed};
    }
    if (!more) break;
    t = t_next;
    r = r_next;
  }
}

// ---------------------------------------------------------------------------
// Span kernel: variable-length keys (offset array) and fixed lengths the tiled
// kernel does not take. One wave (= one workgroup) owns a tile of 64
// consecutive keys, whose bytes are one contiguous span of the packed buffer.
// The span is fetched with fully coalesced 16-B raw buffer loads (1 KiB per
// wave instruction) into registers, staged in LDS, and each lane then hashes
// its own key out of LDS with dword reads funnel-shifted by v_alignbyte_b32
// (keys start at any byte). A tile whose span exceeds the LDS window is hashed
// straight from HBM (wave-uniform fallback; rare for keys <= 311 B).
// One tile per workgroup and as many workgroups as tiles: the hardware
// dispatcher keeps every CU's LDS full of tiles in flight, which measured
// faster than a persistent grid with a one-tile-ahead register prefetch
// (4.42 vs 4.05 TB/s on config D, profiles/r1/ab_span_grid.txt).
// ---------------------------------------------------------------------------
// LDS per workgroup: [0, span) the staged span, then kSpanPad bytes of read
// slack. Variable-length launches take the full window; fixed-length launches
// only what one tile's span needs, so more tiles fit a CU.
constexpr uint32_t kSpanAlloc = 20u * 1024u;                    // 8 workgroups per CU; the most a window takes
constexpr uint32_t kSpanPad = 64;
constexpr uint32_t kSpanCap = kSpanAlloc - kSpanPad;            // 20416 B
constexpr int kSpanPiecesMax = (kSpanCap + 1023u) / 1024u;      // 20

template <bool VAR>
struct SpanTile {
  uint64_t key;       // this lane's key index
  uint64_t start;     // byte offset of this lane's key (relative to `bytes`)
  uint32_t len;       // this lane's key length
  uint32_t valid;     // key < n (not bool: keeps the struct out of scratch when copied)
  uint64_t base;      // absolute address of the span's first 16-B piece (uniform)
  uint32_t span16;    // bytes to stage, multiple of 16 (uniform; > kSpanCap -> fallback)
};

// Raw per-lane offsets of a tile (variable lengths); span_finish turns them
// into the tile's wave-uniform span.
struct SpanRaw {
  uint64_t t;
  uint64_t o0, o1;
};

template <bool VAR>
__device__ __forceinline__ SpanRaw span_load(const uint64_t* offsets, uint64_t n, uint64_t t, uint32_t lane) {
  SpanRaw r;
  r.t = t;
  r.o0 = r.o1 = 0;
  if constexpr (VAR) {
    const uint64_t key = t * 64u + lane;
    if (key < n) {
      r.o0 = offsets[key];
      r.o1 = offsets[key + 1];
    }
  }
  return r;
}

template <bool VAR>
__device__ __forceinline__ SpanTile<VAR> span_finish(const uint8_t* bytes, uint64_t off_base, uint32_t key_len,
                                                     uint64_t n, const SpanRaw& raw, uint32_t lane) {
  SpanTile<VAR> ti;
  const uint64_t k0 = raw.t * 64u;
  const uint32_t kn = (uint32_t)min<uint64_t>(64u, n - k0);
  ti.key = k0 + lane;
  ti.valid = lane < kn;
  uint64_t first, end;  // tile bytes [first, end) relative to `bytes` (wave-uniform)
  if constexpr (VAR) {
    ti.start = raw.o0 - off_base;
    ti.len = (uint32_t)(raw.o1 - raw.o0);
    const uint64_t e_rel = raw.o1 - off_base;
    // the readlane builtins return a signed int: widen through uint32_t, never sign-extend
    first = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)ti.start) |
            ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(ti.start >> 32)) << 32);
    end = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)e_rel, kn - 1) |
          ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(e_rel >> 32), kn - 1) << 32);
  } else {
    ti.start = ti.key * (uint64_t)key_len;
    ti.len = key_len;
    first = k0 * (uint64_t)key_len;
    end = (k0 + kn) * (uint64_t)key_len;
  }
  if (end <= first) {  // every key of the tile is empty: stage and load nothing
    ti.base = 0;
    ti.span16 = 0;
    return ti;
  }
  const uint64_t b = reinterpret_cast<uintptr_t>(bytes);
  ti.base = (b + first) & ~(uint64_t)15;
  const uint64_t span = ((b + end + 15) & ~(uint64_t)15) - ti.base;
  ti.span16 = span > 0xffffffffull ? 0xffffffffu : (uint32_t)span;
  return ti;
}

// Fetch the span into registers: piece q of lane l covers bytes q*1024 + 16l.
// Raw buffer loads through a descriptor whose range is exactly the span: lanes
// past its end get 0 without touching memory, so no per-lane predicate, and no
// load can reach a page the span does not.
template <int PIECES>
__device__ __forceinline__ void span_fetch(u32x4 (&reg)[PIECES], uint64_t base, uint32_t span16, uint32_t lane) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)base);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(base >> 32));
  const uint32_t nb = __builtin_amdgcn_readfirstlane(span16);
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<void*>((uint64_t)lo | ((uint64_t)hi << 32)), (short)0, (int)nb, 0x00020000);
#pragma unroll
  for (int q = 0; q < PIECES; ++q)
    if ((uint32_t)q * 1024u < nb)
      reg[q] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (uint32_t)q * 1024u + lane * 16u, 0, 2 /* nt */);
}

// Stage the fetched pieces that hold span bytes (lanes past the span's end
// write nothing: the window may be exactly the span plus its read slack).
template <int PIECES>
__device__ __forceinline__ void span_stage(uint32_t* lds, const u32x4 (&reg)[PIECES], uint32_t span16,
                                           uint32_t lane) {
#pragma unroll
  for (int q = 0; q < PIECES; ++q)
    if ((uint32_t)q * 1024u < span16 && (uint32_t)q * 1024u + lane * 16u < span16)
      reinterpret_cast<u32x4*>(lds)[64 * q + lane] = reg[q];
}

// The independent k1/k2 mixes (murmurhash3.c:97, :101) of the 16 bytes that
// start `sh` bytes into dwords x0..x4.
__device__ __forceinline__ void mix_dwords(uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3, uint32_t x4,
                                           uint32_t sh, uint64_t& m1, uint64_t& m2) {
  const uint32_t d0 = __builtin_amdgcn_alignbyte(x1, x0, sh);
  const uint32_t d1 = __builtin_amdgcn_alignbyte(x2, x1, sh);
  const uint32_t d2 = __builtin_amdgcn_alignbyte(x3, x2, sh);
  const uint32_t d3 = __builtin_amdgcn_alignbyte(x4, x3, sh);
  m1 = mix_k1(pack64(d0, d1));
  m2 = mix_k2(pack64(d2, d3));
}

// Hash `len` bytes starting at byte offset p of the staged span. Reads may run
// up to 36 (< kSpanPad) bytes past the span, into the window's padding; such
// bytes are never used.
__device__ __forceinline__ State hash_lds(const uint32_t* lds, uint32_t p, uint32_t len, uint32_t seed) {
  const uint32_t sh = p & 3u;
  const uint32_t* w = lds + (p >> 2);
  const uint32_t nblocks = len >> 4;
  State s{seed, seed};
  // Software pipeline over blocks: iteration j runs the serial h1/h2 chain of
  // block j beside the (independent, multiply-heavy) k1/k2 mixes of block j+1,
  // and reads the dwords of block j+2.
  uint32_t a0 = w[0], a1 = w[1], a2 = w[2], a3 = w[3], a4 = w[4];
  uint32_t b1 = w[5], b2 = w[6], b3 = w[7], b4 = w[8];
  uint64_t m1, m2;
  mix_dwords(a0, a1, a2, a3, a4, sh, m1, m2);
  for (uint32_t j = 0; j < nblocks; ++j) {
    const uint32_t* v = w + 4 * j + 8;
    const uint32_t c1 = v[1], c2 = v[2], c3 = v[3], c4 = v[4];
    uint64_t n1, n2;
    mix_dwords(a4, b1, b2, b3, b4, sh, n1, n2);
    chain_block(s, m1, m2);
    m1 = n1;
    m2 = n2;
    a0 = a4;
    a1 = b1;
    a2 = b2;
    a3 = b3;
    a4 = b4;
    b1 = c1;
    b2 = c2;
    b3 = c3;
    b4 = c4;
  }
  uint32_t x0 = a0, x1 = a1, x2 = a2, x3 = a3, x4 = a4;
  const uint32_t rem = len & 15u;
  if (rem) {  // x0..x4 now hold the dwords of the tail
    const uint32_t d0 = __builtin_amdgcn_alignbyte(x1, x0, sh);
    const uint32_t d1 = __builtin_amdgcn_alignbyte(x2, x1, sh);
    const uint32_t d2 = __builtin_amdgcn_alignbyte(x3, x2, sh);
    const uint32_t d3 = __builtin_amdgcn_alignbyte(x4, x3, sh);
    const uint64_t t1 = pack64(d0, d1) & low_bytes_mask(rem);
    const uint64_t t2 = rem > 8 ? (pack64(d2, d3) & low_bytes_mask(rem - 8)) : 0ull;
    tail_block(s, t1, t2, rem);
  }
  finish(s, len);
  return s;
}



// hash_lds with one unaligned ds_read_b128 per block instead of dword reads
// funnel-shifted by v_alignbyte_b32 (gfx950 runs LDS accesses in unaligned
// mode; hipcc emits ds_read_b128 for an align-1 vector LDS load). Variable
// lengths: U[8,512] B keys +4-8 % (profiles/r2/ab_span/).
typedef __attribute__((address_space(3))) const uint8_t lds_u8;
typedef uint32_t u32x4_a1 __attribute__((ext_vector_type(4), aligned(1)));
typedef __attribute__((address_space(3))) const u32x4_a1 lds_u32x4_a1;

__device__ __forceinline__ u32x4 lds_read16(const uint32_t* lds, uint32_t byte) {
  return *(lds_u32x4_a1*)((lds_u8*)lds + byte);  // generic -> LDS address space (lds is an LDS pointer)
}

// Hash `len` bytes at byte offset p of the staged span with one unaligned
// ds_read_b128 per block, in two parts split at the last LDS read: the body
// blocks (hash_lds_u_blocks: the state, and the tail's 16 bytes in `cur`),
// then the register-only tail and finalisation (hash_tail_finish), so a
// window can be handed on between them.
// Software pipeline: block j's chain beside block j+1's mixes and block j+2's
// read (the compiler folds this loop-carried read into one read at the point
// of use; forcing it a block ahead, or a two-block-deep pipeline with block
// j+2's mixes beside block j's chain, measured no faster in k_span or
// k_span_pp: profiles/r2/ab_span/ab_pipe, ab_deep). The read address is the
// loop counter (one VALU add and one compare per block).
__device__ __forceinline__ void hash_lds_u_blocks(const uint32_t* lds, uint32_t p, uint32_t len, uint32_t seed,
                                                  State& s, u32x4& cur) {
  s = State{seed, seed};
  cur = lds_read16(lds, p);
  u32x4 nxt = lds_read16(lds, p + 16u);
  uint64_t m1 = mix_k1(pack64(cur.x, cur.y)), m2 = mix_k2(pack64(cur.z, cur.w));
  // a: the LDS address of nxt
  uint32_t a = (uint32_t)reinterpret_cast<uintptr_t>((lds_u8*)lds + p + 16u);
  const uint32_t end = a + (len & ~15u);
  while (a != end) {
    a += 16u;
    asm("" : "+v"(a));  // keeps the address the only induction variable (LSR would add a counter)
    const u32x4 nn = *(lds_u32x4_a1*)(lds_u8*)(uintptr_t)a;
    const uint64_t n1 = mix_k1(pack64(nxt.x, nxt.y)), n2 = mix_k2(pack64(nxt.z, nxt.w));
    chain_block(s, m1, m2);
    m1 = n1;
    m2 = n2;
    cur = nxt;
    nxt = nn;
  }
}

__device__ __forceinline__ void hash_tail_finish(State& s, const u32x4& cur, uint32_t len) {
  const uint32_t rem = len & 15u;
  if (rem) {  // cur holds the tail's bytes
    const uint64_t t1 = pack64(cur.x, cur.y) & low_bytes_mask(rem);
    const uint64_t t2 = rem > 8 ? (pack64(cur.z, cur.w) & low_bytes_mask(rem - 8)) : 0ull;
    tail_block(s, t1, t2, rem);
  }
  finish(s, len);
}

__device__ __forceinline__ State hash_lds_u(const uint32_t* lds, uint32_t p, uint32_t len, uint32_t seed) {
  State s;
  u32x4 cur;
  hash_lds_u_blocks(lds, p, len, seed, s, cur);
  hash_tail_finish(s, cur, len);
  return s;
}

// ---------------------------------------------------------------------------
// Round kernel: variable-length keys, streamed 128 B per key per round.
// One wave (= one workgroup) owns 64 consecutive keys. Round r stages, for
// every key still running, the 9 aligned 16-B pieces that hold its bytes
// [128r, 128r + 128) (counted from the key's first aligned piece) into a
// 144-B LDS window per key, loaded cooperatively (lane l of load instruction q
// fetches piece (64q + l) % 9 of key (64q + l) / 9: runs of 144 contiguous
// bytes per key), and prefetches round r + 1 into registers while each lane
// hashes its own key's 8 blocks of round r out of its window. LDS per wave is
// ~10 KiB (k_span needs the whole 64-key span, 20 KiB), so twice as many
// tiles are in flight per CU. A tile with a key longer than kVrMaxRounds
// rounds is hashed straight from HBM (hash_bytes).
// ---------------------------------------------------------------------------
constexpr int kVrPieces = 9;                     // 16-B pieces per key per round
constexpr uint32_t kVrWindow = kVrPieces * 16u;  // 144 B
constexpr uint32_t kVrMaxRounds = 64;            // keys up to 8 KiB in the staged path

// Hash the blocks of round r of a key from its LDS window: window bytes
// [sh16, sh16 + 128) are key bytes [128r, 128r + 128). All 36 dwords the
// round can touch are read at once (the k_tiled lesson: ILP over LDS latency),
// the 8 blocks' k1/k2 mixes are computed unconditionally and the chain step is
// kept only for real blocks (no divergent branches); the tail block, if it
// falls in this round, is re-read from the window afterwards.
__device__ __forceinline__ void vround_blocks(State& s, const uint32_t* win, uint32_t sh16, uint32_t first_block,
                                              uint32_t nb, uint32_t rem) {
  const uint32_t sh = sh16 & 3u;
  const uint32_t* w = win + (sh16 >> 2);
  uint32_t x[33];
#pragma unroll
  for (int d = 0; d < 33; ++d) x[d] = w[d];  // up to window byte 3*4 + 32*4 + 3 < 144 + slack
#pragma unroll
  for (uint32_t t = 0; t < 8; ++t) {
    const uint32_t d0 = __builtin_amdgcn_alignbyte(x[4 * t + 1], x[4 * t + 0], sh);
    const uint32_t d1 = __builtin_amdgcn_alignbyte(x[4 * t + 2], x[4 * t + 1], sh);
    const uint32_t d2 = __builtin_amdgcn_alignbyte(x[4 * t + 3], x[4 * t + 2], sh);
    const uint32_t d3 = __builtin_amdgcn_alignbyte(x[4 * t + 4], x[4 * t + 3], sh);
    State n = s;
    body_block(n, pack64(d0, d1), pack64(d2, d3));
    const bool real = first_block + t < nb;
    s.h1 = real ? n.h1 : s.h1;
    s.h2 = real ? n.h2 : s.h2;
  }
  if (rem != 0u && nb >= first_block && nb < first_block + 8u) {
    const uint32_t* v = w + 4u * (nb - first_block);
    const uint32_t y0 = v[0], y1 = v[1], y2 = v[2], y3 = v[3], y4 = v[4];
    const uint32_t d0 = __builtin_amdgcn_alignbyte(y1, y0, sh);
    const uint32_t d1 = __builtin_amdgcn_alignbyte(y2, y1, sh);
    const uint32_t d2 = __builtin_amdgcn_alignbyte(y3, y2, sh);
    const uint32_t d3 = __builtin_amdgcn_alignbyte(y4, y3, sh);
    const uint64_t t1 = pack64(d0, d1) & low_bytes_mask(rem);
    const uint64_t t2 = rem > 8 ? (pack64(d2, d3) & low_bytes_mask(rem - 8)) : 0ull;
    tail_block(s, t1, t2, rem);
  }
}

constexpr uint32_t kVrStageBytes = (64u * kVrPieces + 2u) * 16u;  // windows + read slack
constexpr uint32_t kVrLdsBytes = kVrStageBytes + 2u * 64u * 4u;      // + per-key tables

// Round-streamed hashing of one 64-key tile (this lane: key `key`, bytes
// [start, start + len) of `bytes`). `lds`: kVrLdsBytes, 16-B aligned, private
// to this wave. Wave-uniform control flow.
template <int OUT>
__device__ __forceinline__ void vround_tile(const uint8_t* bytes, uint64_t key, bool valid, uint64_t start,
                                            uint32_t len, uint32_t seed, const Sink& sink, uint8_t* lds) {
  u32x4* stage = reinterpret_cast<u32x4*>(lds);
  uint32_t* s_rel = reinterpret_cast<uint32_t*>(lds + kVrStageBytes);  // key's first aligned piece - tile's
  uint32_t* s_end = s_rel + 64;  // bytes from that piece to the key's end (0: nothing to load)
  const uint32_t lane = __lane_id();
  const uint64_t addr = reinterpret_cast<uintptr_t>(bytes) + start;
  const uint32_t sh16 = (uint32_t)(addr & 15u);
  const uint32_t nb = len >> 4, rem = len & 15u;
  const uint32_t my_rounds = (nb + (rem ? 1u : 0u) + 7u) >> 3;
  uint32_t R = my_rounds;
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) R = max(R, (uint32_t)__shfl_xor((int)R, m));
  R = __builtin_amdgcn_readfirstlane(R);
  State s{seed, seed};
  if (R > kVrMaxRounds) {  // wave-uniform: a key over 8 KiB in this tile
    if (valid) store_result<OUT>(sink, key, hash_bytes(bytes + start, len, seed));
    return;
  }
  // the tile's first aligned piece (lane 0 holds the lowest start; offsets are monotone)
  const uint64_t a16 = addr & ~(uint64_t)15;
  const uint64_t tile0 = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)a16) |
                         ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(a16 >> 32)) << 32);
  s_rel[lane] = (uint32_t)(a16 - tile0);  // < 64 x 8 KiB + 16
  s_end[lane] = len ? sh16 + len : 0u;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // static load mapping: instruction q, lane -> (key lk, piece lp)
  uint32_t lrel[kVrPieces], lend[kVrPieces];
#pragma unroll
  for (int q = 0; q < kVrPieces; ++q) {
    const uint32_t idx = 64u * q + lane;
    const uint32_t lk = idx / kVrPieces, lp = idx % kVrPieces;
    lrel[q] = s_rel[lk] + 16u * lp;
    lend[q] = s_end[lk] > 16u * lp ? s_end[lk] - 16u * lp : 0u;  // bytes left from this piece to the key's end
  }
  // a global (not flat) view: flat loads also count against lgkmcnt, so every
  // LDS wait would drain the prefetch as well
  auto fetch = [&](uint32_t r, u32x4 (&reg)[kVrPieces]) {
#pragma unroll
    for (int q = 0; q < kVrPieces; ++q) {
      reg[q] = u32x4{0u, 0u, 0u, 0u};
      // the piece starts inside the key: its aligned 16 B cannot leave the key's page. Plain
      // (not nt) loads keep lines in L2: the window's last piece is the next round's first
      // (nt: 2.56 vs 1.59 ms at 25M x 260 B, profiles/r1/ab_vround_nt.txt)
      if (128u * r < lend[q]) reg[q] = *reinterpret_cast<g_u32x4*>(tile0 + lrel[q] + 128u * r);
    }
  };
  u32x4 nxt[kVrPieces];
  fetch(0, nxt);
  const uint32_t* win = reinterpret_cast<const uint32_t*>(stage) + lane * (kVrWindow / 4);
  for (uint32_t r = 0; r < R; ++r) {
#pragma unroll
    for (int q = 0; q < kVrPieces; ++q) stage[64 * q + lane] = nxt[q];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (r + 1 < R) fetch(r + 1, nxt);
    if (r < my_rounds) vround_blocks(s, win, sh16, 8u * r, nb, rem);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  finish(s, len);
  if (valid) store_result<OUT>(sink, key, s);
}

template <int OUT>
__global__ __launch_bounds__(64) void k_vround(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ offsets,
                                               uint64_t off_base, uint64_t n, uint32_t seed, Sink sink) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kVrLdsBytes];
  const uint64_t key = (uint64_t)blockIdx.x * 64u + threadIdx.x;
  bool valid = key < n;
  uint64_t start = 0;
  uint32_t len = 0;
  bool bad = false;
  if (valid) {
    const uint64_t o0 = offsets[key], o1 = offsets[key + 1];
    bad = var_key_bad(o0, o1);
    start = o0 - off_base;
    len = (uint32_t)(o1 - o0);
  }
  if (__ballot(bad)) {  // wave-uniform: the tile's span is not trustworthy; per-lane hashing of its good keys
    if (bad) flag_bad_key(sink);
    else if (valid) store_result<OUT>(sink, key, hash_bytes(bytes + start, len, seed));
    return;
  }
  vround_tile<OUT>(bytes, key, valid, start, len, seed, sink, lds);
}

// RFB: a variable-length tile whose span overflows the window is streamed in
// rounds through the window (vround_tile, needs kVrLdsBytes of it); without,
// hashed per lane from HBM (small windows, whose kernel then needs fewer VGPRs).
template <int OUT, bool VAR, int PIECES, bool RFB = true>
__global__ __launch_bounds__(64, 4) void k_span(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ offsets,
                                             uint64_t off_base, uint32_t key_len, uint64_t n, uint32_t seed,
                                             uint32_t cap, Sink sink) {
  extern __shared__ __attribute__((aligned(16))) uint32_t span_lds[];
  const uint32_t lane = threadIdx.x;
  const SpanRaw raw = span_load<VAR>(offsets, n, blockIdx.x, lane);
  if constexpr (VAR) {
    const bool bad = var_key_bad(raw.o0, raw.o1);  // lanes past n carry o0 = o1 = 0
    if (__ballot(bad)) {  // wave-uniform: no span for this tile; per-lane hashing of its good keys
      const uint64_t key = raw.t * 64u + lane;
      if (bad) flag_bad_key(sink);
      else if (key < n) store_result<OUT>(sink, key, hash_bytes(bytes + (raw.o0 - off_base), (uint32_t)(raw.o1 - raw.o0), seed));
      return;
    }
  }
  const SpanTile<VAR> ti = span_finish<VAR>(bytes, off_base, key_len, n, raw, lane);
  if (ti.span16 <= cap) {
    u32x4 reg[PIECES];
    span_fetch<PIECES>(reg, ti.base, ti.span16, lane);
    span_stage<PIECES>(span_lds, reg, ti.span16, lane);
    __syncthreads();
    if (ti.valid) {
      const uint32_t p = (uint32_t)(reinterpret_cast<uintptr_t>(bytes) + ti.start - ti.base);
      // variable lengths: unaligned 16-B reads; fixed lengths keep the dword reads (L = 100, 200, 300 B:
      // 4, 2, 9 % faster that way, profiles/r2/ab_span/)
      store_result<OUT>(sink, ti.key, VAR ? hash_lds_u(span_lds, p, ti.len, seed)
                                                                   : hash_lds(span_lds, p, ti.len, seed));
    }
  } else if constexpr (VAR && RFB) {  // span over the window: stream it in rounds (vround_tile) instead
    vround_tile<OUT>(bytes, ti.key, ti.valid, ti.start, ti.len, seed, sink, reinterpret_cast<uint8_t*>(span_lds));
  } else if (ti.valid) {
    store_result<OUT>(sink, ti.key, hash_bytes(bytes + ti.start, ti.len, seed));
  }
}

// ---------------------------------------------------------------------------
// Ping-pong span kernel (variable-length keys): two waves share one LDS
// window and take turns. Both load their tile's span into registers at once;
// wave 0 stages and hashes its tile while wave 1's span is still arriving,
// then one LDS-only barrier hands the window to wave 1, which stages and
// hashes. A window then holds bytes only while they are
// staged or hashed (one HBM latency per two tiles instead of one per tile),
// and a CU keeps twice as many hashing waves (4 per SIMD) for the same LDS.
// U[8,512] B keys: +10 %, all-260 B: +15 %, U[200,400] B: +12 % over k_span
// (profiles/r2/ab_span/). A tile whose span is over the window is streamed
// through it in rounds (vround_tile) in its wave's turn; a tile with an invalid
// key is hashed per lane straight from HBM.
// (Two or more tiles per wave, each wave loading its next span right after
// its hash, spill past 128 VGPRs; a persistent single-wave variant with the
// next span prefetched into registers during the hash measured 0-10 % slower
// than k_span: neither kept, git history.)
// ---------------------------------------------------------------------------
// Workgroup barrier that waits for this wave's LDS accesses only. (A
// __syncthreads() also waits for every global store in flight, vmcnt(0): in
// k_span_pp that put the round trip of wave 0's result stores between its hash
// and wave 1's, profiles/r2/ab_span/ab_handoff2 vs ab_sort.)
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Orders this wave's LDS writes before its own later LDS reads.
__device__ __forceinline__ void wave_lds_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int OUT>
__device__ __forceinline__ void span_hash_tile(const uint32_t* lds, const uint8_t* bytes, const SpanTile<true>& ti,
                                               uint32_t seed, const Sink& sink) {
  if (ti.valid) {
    const uint32_t p = (uint32_t)(reinterpret_cast<uintptr_t>(bytes) + ti.start - ti.base);
    store_result<OUT>(sink, ti.key, hash_lds_u(lds, p, ti.len, seed));
  }
}

template <int OUT>
__device__ __forceinline__ void span_tile_from_hbm(const uint8_t* bytes, uint64_t off_base, uint64_t n,
                                                   const SpanRaw& raw, uint32_t lane, uint32_t seed, const Sink& sink) {
  const uint64_t key = raw.t * 64u + lane;
  if (var_key_bad(raw.o0, raw.o1)) flag_bad_key(sink);
  else if (key < n)
    store_result<OUT>(sink, key, hash_bytes(bytes + (raw.o0 - off_base), (uint32_t)(raw.o1 - raw.o0), seed));
}

template <int OUT, int PIECES>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(4))) void k_span_pp(
    const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ offsets, uint64_t off_base, uint64_t n,
    uint32_t seed, uint32_t cap, Sink sink) {
  static_assert(OUT != kOutProbe, "the probe's row registers would spill beside the held span: k_span");
  extern __shared__ __attribute__((aligned(16))) uint32_t span_lds[];
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const uint64_t t = 2u * (uint64_t)blockIdx.x + wave;  // this wave's tile (past the last: idle, barriers only)
  const uint64_t ntiles = (n + 63) / 64;
  const bool has = t < ntiles;
  const SpanRaw raw = span_load<true>(offsets, n, t, lane);  // keys past n: o0 = o1 = 0
  const bool bad = __ballot(var_key_bad(raw.o0, raw.o1)) != 0;
  const SpanTile<true> ti = span_finish<true>(bytes, off_base, 0, n, raw, lane);
  const bool staged = has && !bad && ti.span16 <= cap;
  // Wave 0 stages and hashes; one barrier hands the window to wave 1, which
  // stages and hashes in turn (a wave's own LDS writes and reads are ordered
  // by a wave-level fence). One barrier instead of the four of two
  // stage/hash phases: U[8,512] +1.7 %, all-260 B +10.6 %, U[200,400] +4.7 %
  // (profiles/r2/ab_span/ab_handoff2, "t32"). Each wave passes exactly one
  // barrier on either branch; the held span lives only on the staged one, so
  // the round fallback's registers never sit beside it.
  if (staged) {
    u32x4 reg[PIECES];
    span_fetch<PIECES>(reg, ti.base, ti.span16, lane);
    if (wave == 0) {
      span_stage<PIECES>(span_lds, reg, ti.span16, lane);
      wave_lds_fence();
      // the body blocks only: the tail and fmix run after the hand-over, from
      // registers (the state parks in reg[0..1], dead on this wave once staged,
      // so no register is live across the barrier beyond the held span).
      // U[8,512] +1.1-1.5 %, all-260 B +0.9-3.2 %, U[64,448] +0.7-1.6 %
      // (profiles/r3/ab_early_handover*.txt)
      if (ti.valid) {
        State s;
        u32x4 cur;
        hash_lds_u_blocks(span_lds, (uint32_t)(reinterpret_cast<uintptr_t>(bytes) + ti.start - ti.base), ti.len,
                          seed, s, cur);
        reg[0] = u32x4{(uint32_t)s.h1, (uint32_t)(s.h1 >> 32), (uint32_t)s.h2, (uint32_t)(s.h2 >> 32)};
        reg[1] = cur;
      }
    }
    lds_barrier();  // wave 0 has read the window for the last time
    if (wave == 0 && ti.valid) {
      State s{pack64(reg[0].x, reg[0].y), pack64(reg[0].z, reg[0].w)};
      hash_tail_finish(s, reg[1], ti.len);
      store_result<OUT>(sink, ti.key, s);
    }
    if (wave == 1) {
      span_stage<PIECES>(span_lds, reg, ti.span16, lane);
      wave_lds_fence();
      span_hash_tile<OUT>(span_lds, bytes, ti, seed, sink);
    }
  } else {
    // A span over the window is streamed in rounds through this wave's half of
    // it (the round path needs kVrLdsBytes). Wave 0 goes first; wave 1 waits for
    // the hand-over only if wave 0 may be staging a span in the whole window,
    // i.e. unless wave 0's tile is itself over the window (its bytes alone
    // exceed it) -- then both stream at once, as k_vround's independent waves do.
    const bool over = has && !bad;
    uint8_t* win = reinterpret_cast<uint8_t*>(span_lds) + wave * kVrLdsBytes;
    bool first = wave == 0;
    if (wave == 1 && over) {
      const uint64_t s0 = offsets[(t - 1) * 64u];  // wave 0's tile: keys [64 (t - 1), 64 t)
      const uint64_t e0 = pack64(__builtin_amdgcn_readfirstlane((uint32_t)raw.o0),
                                 __builtin_amdgcn_readfirstlane((uint32_t)(raw.o0 >> 32)));
      first = e0 < s0 || e0 - s0 > cap;  // decreasing: wave 0 flags its keys and stages nothing
    }
    if (first && over) vround_tile<OUT>(bytes, ti.key, ti.valid, ti.start, ti.len, seed, sink, win);
    lds_barrier();
    if (!first && over) vround_tile<OUT>(bytes, ti.key, ti.valid, ti.start, ti.len, seed, sink, win);
    if (has && bad) span_tile_from_hbm<OUT>(bytes, off_base, n, raw, lane, seed, sink);
  }
}

// ---------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------
// Pieces (16 B) of every key staged per round by k_tiled. 8 (one 128-B line per
// key per round) when every round is full; otherwise 16, so that a key of
// 12-15 pieces is one round instead of a full and a mostly empty one
// (profiles/r1/sweep_tiled: L=192 5167 GB/s at 16 vs 3689 at 8).
// SHF_HB_TILED_ROUND=4|8|16 overrides it (a tuning knob, read once).
static int tiled_round_pieces(uint32_t key_len) {
  static const int forced = [] {
    const char* e = getenv("SHF_HB_TILED_ROUND");
    const int v = e ? atoi(e) : 0;
    return (v == 4 || v == 8 || v == 16) ? v : 0;
  }();
  if (forced) return forced;
  return ((key_len >> 4) & 7u) == 0 ? 8 : 16;
}

static unsigned grid_for(uint64_t items, unsigned per_block, unsigned cap) {
  uint64_t g = (items + per_block - 1) / per_block;
  if (g > cap) g = cap;
  if (g == 0) g = 1;
  return (unsigned)g;
}

template <int OUT, bool VAR, int PIECES, bool RFB = true>
static hipError_t launch_span_p(const void* bytes, const uint64_t* offsets, uint64_t off_base, uint32_t key_len,
                                uint64_t n, uint32_t seed, const Sink& sink, hipStream_t st, uint32_t lds) {
  const uint64_t tiles = (n + 63) / 64;
  if (tiles > 0x7fffffffull) return hipErrorInvalidValue;  // 137 G keys per launch
  hipLaunchKernelGGL((k_span<OUT, VAR, PIECES, RFB>), dim3((unsigned)tiles), dim3(64), lds, st,
                     reinterpret_cast<const uint8_t*>(bytes), offsets, off_base, key_len, n, seed, lds - kSpanPad,
                     sink);
  return hipGetLastError();
}

// LDS window per 64-key tile of a variable-length batch. Unknown byte count:
// 20 KiB (8 tiles per CU; config D's U[8,512] spans average 16.6 KB). Known
// (key_bytes = offsets[n] - offsets[0]): at least the tile's expected span,
// 64 x the mean key length, plus a tenth and 512 B; then grown to the most LDS
// per tile that keeps as many tiles per CU (the LDS and register limits) and
// that the instantiation's PIECES 1-KiB fetches cover. A CU holds 160 KiB /
// window tiles, and a tile's window only loads while its span is in flight:
// smaller windows keep more spans in flight (U[8,128] keys: 5.17 vs 3.39 TB/s
// at 10 vs 20 KiB, profiles/r1/ab_window/, ab_sized/).
constexpr uint32_t kLdsPerCu = 160u * 1024u;

// Ping-pong span kernel: one 128-thread workgroup per two tiles, one window.
template <int OUT>
static hipError_t launch_var_span_pingpong(const void* bytes, const uint64_t* offsets, uint64_t off_base, uint64_t n,
                                           uint32_t seed, const Sink& sink, hipStream_t st) {
  static_assert(kSpanAlloc - kSpanPad >= 2u * kVrLdsBytes && kVrLdsBytes % 16u == 0,
                "the window holds two waves' round fallback LDS");
  const uint64_t tiles = (n + 63) / 64;
  const uint64_t wgs = (tiles + 1) / 2;
  if (wgs > 0x7fffffffull) return hipErrorInvalidValue;
  hipLaunchKernelGGL((k_span_pp<OUT, kSpanPiecesMax>), dim3((unsigned)wgs), dim3(128), kSpanAlloc, st,
                     reinterpret_cast<const uint8_t*>(bytes), offsets, off_base, n, seed, kSpanAlloc - kSpanPad, sink);
  return hipGetLastError();
}

template <int OUT, int PIECES, bool RFB>
static hipError_t launch_var_span(const void* bytes, const uint64_t* offsets, uint64_t off_base, uint64_t n,
                                  uint32_t seed, const Sink& sink, hipStream_t st, uint32_t need) {
  static const uint32_t reg_tiles = [] {  // tiles per CU the kernel's registers allow
    int b = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, reinterpret_cast<const void*>(&k_span<OUT, true, PIECES, RFB>),
                                                     64, 0) != hipSuccess || b < 1)
      b = 1;
    return (uint32_t)b;
  }();
  const uint32_t top = std::min<uint32_t>((uint32_t)PIECES * 1024u + kSpanPad, kSpanAlloc);
  uint32_t tiles = std::min<uint32_t>(kLdsPerCu / need, reg_tiles);
  if (tiles < 1) tiles = 1;
  uint32_t lds = (kLdsPerCu / tiles) & ~255u;
  lds = std::min(std::max(lds, need), top);
  return launch_span_p<OUT, true, PIECES, RFB>(bytes, offsets, off_base, 0, n, seed, sink, st, lds);
}

// Fixed lengths: a tile's span is at most 64 * key_len + 15 bytes, so the LDS
// request (and the fetch) is sized to that; variable lengths use the window.
// pingpong: AUTO may take k_span_pp (a forced SHF_HB_KERNEL_SPAN keeps k_span).
template <int OUT, bool VAR>
static hipError_t launch_span(const void* bytes, const uint64_t* offsets, uint64_t off_base, uint32_t key_len,
                              uint64_t n, uint32_t seed, const Sink& sink, hipStream_t st, uint64_t key_bytes = 0,
                              bool pingpong = false) {
  if constexpr (VAR) {
    const double need = key_bytes && n ? 64.0 * (double)key_bytes / (double)n * 1.1 + 512.0 + kSpanPad : 1e30;
    // windows over 10 KiB (config D's U[8,512] B keys) or an unknown byte count: two waves per
    // window, overflowing tiles streamed in rounds through it
    if constexpr (OUT != kOutProbe)
      if (pingpong && need > 10240.0 + kSpanPad)
        return launch_var_span_pingpong<OUT>(bytes, offsets, off_base, n, seed, sink, st);
    if (need >= (double)kSpanAlloc)
      return launch_span_p<OUT, VAR, kSpanPiecesMax>(bytes, offsets, off_base, 0, n, seed, sink, st, kSpanAlloc);
    const uint32_t w = (uint32_t)need;
    // (PIECES 6 and 8 spill to scratch under hipcc 7.2; 4 and 10 take 55 and 47 VGPRs: 8 waves per SIMD)
    if (w <= 4096u + kSpanPad) return launch_var_span<OUT, 4, false>(bytes, offsets, off_base, n, seed, sink, st, w);
    if (w <= 10240u + kSpanPad) return launch_var_span<OUT, 10, false>(bytes, offsets, off_base, n, seed, sink, st, w);
    static_assert(10240u + kSpanPad >= kVrLdsBytes, "windows with the round fallback hold its LDS");
    return launch_var_span<OUT, kSpanPiecesMax, true>(bytes, offsets, off_base, n, seed, sink, st, w);
  } else {
    const uint32_t span = ((uint32_t)key_len * 64u + 15u + 15u) & ~15u;
    const uint32_t lds = (span + kSpanPad + 255u) & ~255u;
    // (a PIECES = 8 instantiation spills to scratch under hipcc 7.2: use 4 or 20)
    if (span <= 4096) return launch_span_p<OUT, VAR, 4>(bytes, offsets, off_base, key_len, n, seed, sink, st, lds);
    return launch_span_p<OUT, VAR, kSpanPiecesMax>(bytes, offsets, off_base, key_len, n, seed, sink, st, lds);
  }
}

template <int OUT>
static hipError_t launch_fixed_t(const void* keys, uint32_t key_len, uint64_t n, uint32_t seed, const Sink& sink,
                                 hipStream_t st, int kernel) {
  const bool al16 = (reinterpret_cast<uintptr_t>(keys) & 15u) == 0;
  if (kernel == kKernelAuto) {
    // Measured on MI355X, 6.4 GB batches (tools/sweep_fixed.sh, tools/sweep_tiled*.sh,
    // profiles/r1/sweep_fixed_v2, profiles/r1/sweep_tiled):
    //  - k_tiled (8 pieces per round) when every round is full: key_len % 128 == 0;
    //  - k_span for lengths whose 64-key tiles fit its LDS window, except
    //    multiples of 64 B, whose lane-per-key LDS reads all hit the same banks
    //    (L=144..240: 5191-5680 GB/s against 4871-5423 for k_tiled<16>);
    //  - k_tiled (16 pieces per round) when its one partial round is >= 3/4 full
    //    (L=192: 5167 against generic 4564, span 4197);
    //  - short keys (< 48 B) and the rest: per-lane loads (k_generic).
    const uint32_t pieces = key_len >> 4;
    const bool whole16 = (key_len & 15u) == 0 && al16;
    if (key_len == 16 && al16) kernel = kKernelFixed16;
    else if (whole16 && key_len >= 128 && (pieces & 7u) == 0) kernel = kKernelTiled;
    else if (key_len >= 48 && (key_len & 63u) != 0 && (uint64_t)key_len * 64u + 16u <= kSpanCap)
      kernel = kKernelSpan;
    else if (whole16 && key_len >= 128 && (pieces & 15u) >= 12) kernel = kKernelTiled;
    else kernel = kKernelGeneric;
  }
  switch (kernel) {
    case kKernelFixed16:
    {
      constexpr uint64_t per_block = kF16Block;
      if (key_len != 16 || !al16 || (n + per_block - 1) / per_block > 0x7fffffffull) return hipErrorInvalidValue;
      hipLaunchKernelGGL(k_fixed16<OUT>, dim3((unsigned)((n + per_block - 1) / per_block)), dim3(kF16Block), 0, st,
                         reinterpret_cast<const u32x4*>(keys), n, seed, sink);
    }
      break;
    case kKernelTiled: {
      if (key_len < 32 || (key_len & 15u) || !al16) return hipErrorInvalidValue;
      const uint64_t tiles = (n + kTileKeys - 1) / kTileKeys;
      const int r = tiled_round_pieces(key_len);
      const dim3 g(grid_for(tiles, kTiledWaves, 0xffffffffu)), b(64 * kTiledWaves);
      const uint8_t* k8 = reinterpret_cast<const uint8_t*>(keys);
      if (r == 4) hipLaunchKernelGGL((k_tiled<OUT, 4>), g, b, 0, st, k8, key_len, n, seed, sink);
      else if (r == 16) hipLaunchKernelGGL((k_tiled<OUT, 16>), g, b, 0, st, k8, key_len, n, seed, sink);
      else hipLaunchKernelGGL((k_tiled<OUT, 8>), g, b, 0, st, k8, key_len, n, seed, sink);
      break;
    }
    case kKernelSpan:
      return launch_span<OUT, false>(keys, nullptr, 0, key_len, n, seed, sink, st);
    default:
      hipLaunchKernelGGL((k_generic<OUT, false>), dim3(grid_for(n, 256, kGenericGridCap)), dim3(256), 0, st,
                         reinterpret_cast<const uint8_t*>(keys), (const uint64_t*)nullptr, (uint64_t)0, key_len, n,
                         seed, sink);
      break;
  }
  return hipGetLastError();
}

template <int OUT>
static hipError_t launch_var_t(const void* bytes, const uint64_t* offsets, uint64_t off_base, uint64_t n,
                               uint32_t seed, const Sink& sink, hipStream_t st, int kernel, uint64_t key_bytes) {
  // AUTO with a known byte count: the span kernel with a sized window up to a
  // mean key length of 300 B; beyond, 64-key spans overflow even 20 KiB and the
  // round kernel streams them (profiles/r1/sweep_var: U[8,2048] round 3797,
  // span 3247 GB/s).
  if (kernel == kKernelAuto && key_bytes != 0 && key_bytes / n > 300) kernel = kKernelRound;
  if (kernel == kKernelGeneric) {
    hipLaunchKernelGGL((k_generic<OUT, true>), dim3(grid_for(n, 256, kGenericGridCap)), dim3(256), 0, st,
                       reinterpret_cast<const uint8_t*>(bytes), offsets, off_base, (uint32_t)0, n, seed, sink);
    return hipGetLastError();
  }
  if (kernel == kKernelRound) {
    const uint64_t tiles = (n + 63) / 64;
    if (tiles > 0x7fffffffull) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_vround<OUT>, dim3((unsigned)tiles), dim3(64), 0, st, reinterpret_cast<const uint8_t*>(bytes),
                       offsets, off_base, n, seed, sink);
    return hipGetLastError();
  }
  if (kernel == kKernelSpanPP) {
    if constexpr (OUT == kOutProbe) return hipErrorInvalidValue;
    else return launch_var_span_pingpong<OUT>(bytes, offsets, off_base, n, seed, sink, st);
  }
  return launch_span<OUT, true>(bytes, offsets, off_base, 0, n, seed, sink, st, key_bytes, kernel == kKernelAuto);
}

hipError_t launch_fixed(const void* keys, uint32_t key_len, uint64_t n, uint32_t seed, const Sink& sink,
                        int out_mode, hipStream_t st, int kernel) {
  if (n == 0) return hipSuccess;
  switch (out_mode) {
    case kOutHash:
      return launch_fixed_t<kOutHash>(keys, key_len, n, seed, sink, st, kernel);
    case kOutUid:
      return launch_fixed_t<kOutUid>(keys, key_len, n, seed, sink, st, kernel);
    case kOutHashWin: {
      bool ranked = false;
      return launch_fixed_win(keys, key_len, n, seed, sink, st, kernel, &ranked);
    }
    case kOutUidWin:
      return launch_fixed_t<kOutUidWin>(keys, key_len, n, seed, sink, st, kernel);
    default:
      return launch_fixed_t<kOutProbe>(keys, key_len, n, seed, sink, st, kernel);
  }
}

hipError_t launch_fixed_win(const void* keys, uint32_t key_len, uint64_t n, uint32_t seed, const Sink& sink,
                            hipStream_t st, int kernel, bool* ranked) {
  *ranked = false;
  if (n == 0) return hipSuccess;
  const bool al16 = (reinterpret_cast<uintptr_t>(keys) & 15u) == 0;
  if (key_len == 16 && al16 && sink.win_counts && sink.win_sorted &&
      (kernel == kKernelAuto || kernel == kKernelFixed16)) {
    const uint64_t chunks = (n + kWoChunk - 1) / kWoChunk;
    if (chunks > 0x7fffffffull) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_fixed16_win<kF16WinBlock>, dim3((unsigned)chunks), dim3(kF16WinBlock), 0, st,
                       reinterpret_cast<const u32x4*>(keys), n, seed, sink);
    *ranked = true;
    return hipGetLastError();
  }
  return launch_fixed_t<kOutHashWin>(keys, key_len, n, seed, sink, st, kernel);
}

hipError_t launch_var(const void* bytes, const uint64_t* offsets, uint64_t off_base, uint64_t n, uint32_t seed,
                      const Sink& sink, int out_mode, hipStream_t st, int kernel, uint64_t key_bytes) {
  if (n == 0) return hipSuccess;
  switch (out_mode) {
    case kOutHash:
      return launch_var_t<kOutHash>(bytes, offsets, off_base, n, seed, sink, st, kernel, key_bytes);
    case kOutUid:
      return launch_var_t<kOutUid>(bytes, offsets, off_base, n, seed, sink, st, kernel, key_bytes);
    case kOutHashWin:
      return launch_var_t<kOutHashWin>(bytes, offsets, off_base, n, seed, sink, st, kernel, key_bytes);
    case kOutUidWin:
      return launch_var_t<kOutUidWin>(bytes, offsets, off_base, n, seed, sink, st, kernel, key_bytes);
    default:
      return launch_var_t<kOutProbe>(bytes, offsets, off_base, n, seed, sink, st, kernel, key_bytes);
  }
}

__global__ __launch_bounds__(64) void k_status_take(uint32_t* word, uint32_t* taken) {
  if (threadIdx.x == 0) *taken = atomicExch(word, 0u);
}

hipError_t launch_status_take(uint32_t* word, uint32_t* taken, hipStream_t st) {
  hipLaunchKernelGGL(k_status_take, dim3(1), dim3(64), 0, st, word, taken);
  return hipGetLastError();
}

// One workgroup per window: its 2048 entries' distinct indexed values are
// inserted into an LDS hash table, ranked in table order (a block scan), and
// each entry is replaced by its value's rank.
constexpr uint32_t kMapTable = 4096;  // >= 2 x 2048: open addressing stays short

__global__ __launch_bounds__(256) void k_compact_map(const uint32_t* __restrict__ tab_slot, uint64_t n_slots,
                                                     uint8_t* __restrict__ map8, uint32_t* __restrict__ win_tab) {
  __shared__ uint32_t key[kMapTable];
  __shared__ uint32_t rank[kMapTable];
  __shared__ uint32_t wsum[4];
  const uint32_t win = blockIdx.x, t = threadIdx.x, lane = t & 63u, wave = t >> 6;
  for (uint32_t i = t; i < kMapTable; i += 256) key[i] = kProbeNone;
  __syncthreads();
  uint32_t e[8];
#pragma unroll
  for (uint32_t j = 0; j < 8; ++j) {
    e[j] = tab_slot[(win << 11) + j * 256u + t];
    if (e[j] != kProbeNone && (uint64_t)(e[j] >> 11) >= n_slots) e[j] = kProbeNone;  // not indexed
    if (e[j] == kProbeNone) continue;
    for (uint32_t h = (e[j] * 0x9e3779b1u) >> 20;; h = (h + 1) & (kMapTable - 1)) {
      const uint32_t old = atomicCAS(&key[h], kProbeNone, e[j]);
      if (old == kProbeNone || old == e[j]) break;
    }
  }
  __syncthreads();
  // ranks in table order: thread t owns table entries [16 t, 16 t + 16)
  uint32_t cnt = 0;
#pragma unroll
  for (uint32_t i = 0; i < 16; ++i) cnt += key[16 * t + i] != kProbeNone;
  uint32_t incl = cnt;
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t v = __shfl_up(incl, d);
    if (lane >= d) incl += v;
  }
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  uint32_t r = incl - cnt;
  for (uint32_t w = 0; w < wave; ++w) r += wsum[w];
#pragma unroll
  for (uint32_t i = 0; i < 16; ++i) {
    const uint32_t h = 16 * t + i;
    if (key[h] == kProbeNone) continue;
    rank[h] = r;
    if (r < kMapRanks) win_tab[(win << 8) + r] = key[h];
    ++r;
  }
  __syncthreads();
#pragma unroll
  for (uint32_t j = 0; j < 8; ++j) {
    uint32_t m = kMapNone;
    if (e[j] != kProbeNone) {
      uint32_t h = (e[j] * 0x9e3779b1u) >> 20;
      while (key[h] != e[j]) h = (h + 1) & (kMapTable - 1);
      m = rank[h] < kMapRanks ? rank[h] : kMapEscape;
    }
    map8[(win << 11) + j * 256u + t] = (uint8_t)m;
  }
}

hipError_t launch_compact_map(const uint32_t* tab_slot, uint64_t n_slots, uint8_t* map8, uint32_t* win_tab,
                              hipStream_t st) {
  hipLaunchKernelGGL(k_compact_map, dim3(256), dim3(256), 0, st, tab_slot, n_slots, map8, win_tab);
  return hipGetLastError();
}

hipError_t launch_probe_hashes(const void* hashes, uint64_t n, const Sink& sink, hipStream_t st) {
  if (n == 0) return hipSuccess;
  if ((n + 255) / 256 > 0x7fffffffull) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_probe_hashes, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                     reinterpret_cast<const u32x4*>(hashes), n, sink);
  return hipGetLastError();
}

}  // namespace shfhb
