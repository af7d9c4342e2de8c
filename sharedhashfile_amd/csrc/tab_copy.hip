// Device tab part / shrink copy.
//
// The reference re-packs a tab's key,value data in two places:
//   shf_tab_part()   /root/reference/src/shf.c:722-779 -- after the window's
//                    tab2 -> tab map sends every second tab2 of a full tab to a
//                    new tab (:683-692), every ref whose tab2 now names the new
//                    tab is copied into it (SHF_TAB_REF_COPY, :633-651, appending
//                    with SHF_TAB_APPEND, :545-610), then
//   shf_tab_shrink() /root/reference/src/shf.c:678-720 -- the old tab is
//                    re-created and every remaining ref copied into it.
// Both outputs are fresh tabs filled by appends in row/ref order, so a tab
// image splits in one pass: a ref's record goes to the "move" image (its tab2
// names tab_new) or the "keep" image, at the running sum of the record sizes
// before it in that image; its ref keeps its row and slot.
//
// One 512-thread workgroup per tab (a job). Record lengths: on packed tabs
// (no deleted record) the distance from each record's position to the next
// one's, the 8192 positions bucket-sorted in LDS; otherwise each record's two
// length words. The refs then go in four segments of 2048 (thread t: refs
// t + 512 j of each): DPP wave scans of the record sizes per output image,
// the 8 wave totals through LDS, each ref's row entry written into both
// images and its record's (end, position) appended to that image's list in
// LDS, then the data chunks the segment completes are copied (copy_chunks:
// 16-B destination chunks on consecutive lanes, coalesced full-line stores).
// The headers' tab_size is a closed form when no record times the growth
// factor exceeds a page, else two waves replay SHF_TAB_APPEND's growth
// (:562-565) with a wave-wide forward search of the scanned ends.
// HBM: each record is read once and written once, the 64-KiB rows are read
// once (twice on packed tabs, the second from cache) and written twice.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/shf_hash_batch.h"
#include "kernels.h"

namespace shfhb {

namespace {

constexpr uint32_t kTabHdr = 24;                          // 6 x u32 (shf.private.h:59-65)
constexpr uint32_t kTabRefs = 512 * 16;                   // SHF_ROWS_PER_TAB x SHF_REFS_PER_ROW
constexpr uint32_t kTabData = kTabHdr + kTabRefs * 8;     // offsetof(SHF_TAB_MMAP, data) = 65560
constexpr uint32_t kPage = 4096;                          // SHF_SIZE_PAGE
constexpr uint32_t kThreads = 512;  // one row per thread (1024 measured no faster)
constexpr uint32_t kWaves = kThreads / 64;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4_a1 __attribute__((ext_vector_type(4), aligned(1)));
typedef uint32_t u32_a1 __attribute__((aligned(1)));
typedef uint64_t u64_a1 __attribute__((aligned(1)));
typedef uint16_t u16_a1 __attribute__((aligned(1)));

__device__ __forceinline__ uint64_t mod_page(uint64_t b) { return ((b - 1) / kPage + 1) * kPage; }  // shf.defines.h:76

// Unaligned little-endian u32 of global memory (records start at any byte;
// gfx950 global accesses are unaligned-capable).
__device__ __forceinline__ uint32_t load_u32(const uint8_t* p) { return *reinterpret_cast<const u32_a1*>(p); }

__device__ __forceinline__ void store_u32(uint8_t* p, uint32_t v) { *reinterpret_cast<u32_a1*>(p) = v; }

// Bytes [0, n) of v (n < 16) to p, exactly: 8-, 4-, 2- and 1-byte stores.
__device__ __forceinline__ void store_partial(uint8_t* p, u32x4 v, uint32_t n) {
  uint32_t o = 0;
  uint64_t lo = (uint64_t)v.x | ((uint64_t)v.y << 32), hi = (uint64_t)v.z | ((uint64_t)v.w << 32);
  if (n & 8) {
    *reinterpret_cast<u64_a1*>(p) = lo;
    lo = hi;
    o = 8;
  }
  if (n & 4) {
    *reinterpret_cast<u32_a1*>(p + o) = (uint32_t)lo;
    lo >>= 32;
    o += 4;
  }
  if (n & 2) {
    *reinterpret_cast<u16_a1*>(p + o) = (uint16_t)lo;
    lo >>= 16;
    o += 2;
  }
  if (n & 1) p[o] = (uint8_t)lo;
}

// Wave-wide inclusive scan of a u32 (DPP: shifts by 1, 2, 4, 8 lanes within
// each row of 16, then rows 0 and 1's last lanes added into the rows after
// them; six VALU adds, no ds_bpermute; +7.5 % over a __shfl_up scan).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);  // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);  // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);  // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true);  // row_shr:8
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15 into rows 1, 3
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31 into rows 2, 3
  return v;
}

// One image's records in image order, in LDS: rank r at e[base + dir * r] (the
// keep image's list grows up from 0, the move image's down from the top, so
// the two never meet: a tab has at most 8192 records). end(r) = the record's
// end in the image's data, pos(r) = its byte in the source image.
struct RecList {
  const uint32_t* e_end;
  const uint32_t* e_pos;
  int32_t base, dir;
  __device__ uint32_t end(uint32_t r) const { return e_end[base + dir * (int32_t)r]; }
  __device__ uint32_t pos(uint32_t r) const { return e_pos[base + dir * (int32_t)r]; }
};

// tab_size after appending an image's records in order to a fresh tab
// (SHF_GET_TAB_MMAP's initial size MOD_PAGE(sizeof(SHF_TAB_MMAP)), then
// SHF_TAB_APPEND's growth MOD_PAGE(tab_size + data_needed * factor) whenever a
// record does not fit). ends[0..n) = data bytes up to and including each of
// the image's records (increasing). One wave; every lane returns the size.
// The first record whose end exceeds the room is found 64 ends at a time,
// moving forward only.
__device__ uint64_t replay_tab_size(const RecList& L, uint32_t n, uint32_t factor, uint32_t lane) {
  uint64_t size = mod_page(kTabData);
  uint32_t i0 = 0;
  for (;;) {
    const uint64_t room = size - kTabData;
    uint64_t hit = 0;
    while (i0 < n) {
      hit = __ballot(i0 + lane < n && (uint64_t)L.end(i0 + lane) > room);
      if (hit) break;
      i0 += 64;
    }
    if (!hit) return size;
    i0 += (uint32_t)__builtin_ctzll(hit);  // first record that does not fit
    const uint32_t len = L.end(i0) - (i0 ? L.end(i0 - 1) : 0u);
    size = mod_page(size + (uint64_t)len * factor);
  }
}

// 16 bytes of the source image at `at` (the last piece of the image is read
// byte by byte: no access past its end).
__device__ __forceinline__ unsigned __int128 load16(const uint8_t* src, uint64_t src_len, uint64_t at) {
  if (at + 16u <= src_len) {
    const u32x4 v = *reinterpret_cast<const u32x4_a1*>(src + at);
    return (unsigned __int128)v.x | ((unsigned __int128)v.y << 32) | ((unsigned __int128)v.z << 64) |
           ((unsigned __int128)v.w << 96);
  }
  unsigned __int128 r = 0;
  for (uint32_t i = 0; at + i < src_len && i < 16u; ++i) r |= (unsigned __int128)src[at + i] << (8 * i);
  return r;
}

__device__ __forceinline__ void flag(shf_tab_job* job, int v) {
  *reinterpret_cast<volatile int32_t*>(&job->status) = v;
}

constexpr uint32_t kChunksPerLane = 2;  // 16-B chunks per lane in flight (2 and 4 within 5 %, 8 slower: profiles/r2/ab_tab)

// The first of L's n records whose end lies past x (n if none), x
// wave-uniform: a 64-ary search, each round every lane probes one end and a
// ballot narrows the range 64-fold (8192 records: 3 rounds of one LDS read).
__device__ __forceinline__ uint32_t wave_first_end_past(const RecList& L, uint32_t n, uint32_t x, uint32_t lane) {
  uint32_t lo = 0, span = n;  // the answer lies in [lo, lo + span]
  while (span > 0) {
    const uint32_t step = (span + 63u) >> 6, hi = lo + span;
    const uint32_t p = lo + step * (lane + 1u) - 1u;
    const uint64_t m = __ballot(p >= hi || L.end(p) > x);
    const uint32_t f = m ? (uint32_t)__builtin_ctzll(m) : 64u;
    lo = __builtin_amdgcn_readfirstlane(min(lo + step * f, hi));
    span = __builtin_amdgcn_readfirstlane(min(step - 1u, hi - lo));
  }
  return lo;
}

// out with its bytes from sp on taken from x, byte sp replaced by type (a
// record starting there: its SHF_DATA_TYPE).
__device__ __forceinline__ unsigned __int128 put_at(unsigned __int128 out, unsigned __int128 x, uint32_t sp,
                                                   uint32_t type) {
  const uint32_t sh = 8u * (sp & 7u);
  const uint64_t ones = ~0ull << sh, eq = 0xffull << sh, tv = (uint64_t)type << sh;
  uint64_t ol = (uint64_t)out, oh = (uint64_t)(out >> 64);
  const uint64_t xl = (uint64_t)x, xh = (uint64_t)(x >> 64);
  if (sp < 8u) {
    ol = (ol & ~ones) | (xl & ones & ~eq) | tv;
    oh = xh;
  } else {
    oh = (oh & ~ones) | (xh & ones & ~eq) | tv;
  }
  return ((unsigned __int128)oh << 64) | ol;
}

// Copy the image's data chunks [c_begin, c_end) (absolute 16-B chunks; the
// image's data starts at absolute byte d0 and its records [0, nrec) are in L,
// `total` bytes of them): consecutive chunks on consecutive lanes of the
// workgroup, kChunksPerLane per lane in flight. A chunk takes its bytes from
// the record holding its first byte and the next ones where it crosses a
// record end, each loaded 16 B at the address that puts its bytes at their
// chunk positions, then merged by byte masks (put_at); a record's first byte
// is its SHF_DATA_TYPE, written as the job says (shf.c:593-596). Only the
// data's bytes are written (a chunk straddling its start or end is stored
// partially).
//
// A chunk's record: each wave holds 64 consecutive chunks, so one 64-ary
// search finds the record of its first chunk (r0), every lane loads the end
// of record r0 + lane and counts it into the histogram `hist` (this wave's 64
// words of LDS) at the first chunk lane that reaches it; the inclusive scan
// of the histogram is then each chunk's record - r0 (a chunk 64 or more
// records on, from records under 16 B, falls back to a binary search).
__device__ void copy_chunks(const uint8_t* src, uint64_t src_len, const RecList& L, uint32_t nrec, uint64_t total,
                            uint64_t d0, uint64_t c_begin, uint64_t c_end, uint32_t type, uint32_t t,
                            uint32_t* hist) {
  constexpr uint32_t Q = kChunksPerLane;
  for (uint64_t base = c_begin; base < c_end; base += Q * kThreads) {
    unsigned __int128 v[Q];
    unsigned __int128 vn[Q];  // the next record's first bytes, for a chunk that crosses into it
    uint32_t k[Q], lo[Q], hi[Q], st[Q];
    int64_t a[Q];
#pragma unroll
    for (uint32_t q = 0; q < Q; ++q) {
      const uint64_t c = base + q * kThreads + t;
      a[q] = (int64_t)(c << 4) - (int64_t)d0;  // the chunk's first byte in the image's data
      lo[q] = a[q] < 0 ? 0u : (uint32_t)a[q];
      hi[q] = c < c_end ? (uint32_t)min<int64_t>(a[q] + 16, (int64_t)total) : lo[q];
      uint32_t l = 0, h = nrec;  // first record ending past lo: in [l, h)
      if (__ballot(lo[q] < hi[q])) {  // lane 0 holds the wave's first chunk, active if any is
        const uint32_t lane = t & 63u;
        const uint32_t r0 = wave_first_end_past(L, nrec, __builtin_amdgcn_readfirstlane(lo[q]), lane);
        const uint32_t e = r0 + lane < nrec ? L.end(r0 + lane) : 0xffffffffu;
        hist[lane] = 0;
        __builtin_amdgcn_wave_barrier();
        // e > lane 0's lo, so the first chunk lane whose lo reaches e is >= 1
        const int64_t a0 = a[q] - 16 * (int64_t)lane;
        const int64_t first = ((int64_t)e - a0 + 15) >> 4;
        if (e != 0xffffffffu && first < 64) atomicAdd(&hist[(uint32_t)first], 1u);
        __builtin_amdgcn_wave_barrier();
        const uint32_t cnt = wave_incl_scan(hist[lane]);
        __builtin_amdgcn_wave_barrier();
        if (cnt < 64u) l = h = r0 + cnt;
        else l = r0 + 64u;
      }
      if (lo[q] >= hi[q]) h = l;  // nothing to copy: no search
      while (l < h) {
        const uint32_t mid = (l + h) >> 1;
        if (L.end(mid) > lo[q]) h = mid;
        else l = mid + 1;
      }
      k[q] = l;
      if (lo[q] < hi[q]) {
        st[q] = l ? L.end(l - 1) : 0u;
        // loaded so that byte i of each value is the chunk's byte i (the bytes
        // before a record, or before the image's data, are never stored)
        const uint32_t e = L.end(l);
        v[q] = load16(src, src_len, (uint64_t)((int64_t)L.pos(l) + a[q] - (int64_t)st[q]));
        vn[q] = e < hi[q] ? load16(src, src_len, (uint64_t)((int64_t)L.pos(l + 1) + a[q] - (int64_t)e))
                          : (unsigned __int128)0;
      }
    }
#pragma unroll
    for (uint32_t q = 0; q < Q; ++q) {
      if (lo[q] >= hi[q]) continue;
      const uint32_t s0 = (uint32_t)((int64_t)lo[q] - a[q]);
      unsigned __int128 out = v[q], x = vn[q];
      if (st[q] == lo[q]) out = put_at(out, out, s0, type);  // the record starts at the chunk's first byte
      for (uint32_t kk = k[q], b = L.end(kk); b < hi[q];) {  // record kk + 1 starts at chunk byte b - a
        out = put_at(out, x, (uint32_t)((int64_t)b - a[q]), type);
        const uint32_t e = L.end(++kk);
        if (e < hi[q]) x = load16(src, src_len, (uint64_t)((int64_t)L.pos(kk + 1) + a[q] - (int64_t)e));
        b = e;
      }
      uint8_t* dst = reinterpret_cast<uint8_t*>((base + q * kThreads + t) << 4);
      const uint32_t n = hi[q] - lo[q];  // bytes written, from chunk byte s0
      if (n == 16u) {
        *reinterpret_cast<u32x4*>(dst) =
            u32x4{(uint32_t)out, (uint32_t)(out >> 32), (uint32_t)(out >> 64), (uint32_t)(out >> 96)};
      } else {
        const unsigned __int128 y = out >> (8 * s0);
        store_partial(dst + s0, u32x4{(uint32_t)y, (uint32_t)(y >> 32), (uint32_t)(y >> 64), (uint32_t)(y >> 96)}, n);
      }
    }
  }
}

}  // namespace

// Segments of refs processed in order: each reads its refs' length words and
// copies its records while the lines those reads pulled in are still in L2 /
// the Infinity Cache (one pass over the whole tab's lengths first would evict
// them before the copy at 2 tabs per CU: the data are read twice from HBM).
constexpr uint32_t kSegs = 4;  // 2, 8 and 16 segments measured slower (profiles/r2/ab_tab)
constexpr uint32_t kSegRefs = kTabRefs / kSegs;           // 2048
constexpr uint32_t kSlabs = kSegRefs / kThreads;          // 4: ref = seg * 2048 + slab * 512 + thread

// The segment loop's barriers guard LDS only (the scan sums, the record
// lists, `bad`): wait for this wave's LDS accesses, not for its row and chunk
// stores still in flight as __syncthreads() would (vmcnt(0)).
__device__ __forceinline__ void seg_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4))) void k_tab_split(const uint8_t* __restrict__ src_base, uint64_t src_bytes,
                                                        uint8_t* dst_base, uint64_t dst_bytes, shf_tab_job* jobs,
                                                        const uint16_t* __restrict__ maps, uint32_t n_maps,
                                                        shf_tab_params prm) {
  __shared__ uint32_t e_end[kTabRefs];  // both images' record lists (RecList)
  __shared__ uint32_t e_pos[kTabRefs];
  __shared__ uint32_t wsum[2][kSlabs][4][kWaves];  // per segment parity, slab, quantity (keep/move bytes/refs), wave
  __shared__ int bad;
  __shared__ uint32_t max_len;  // the longest record copied (either image)
  __shared__ unsigned long long len_total;  // every record length so far, exactly (u64)
  __shared__ uint32_t wtot[kWaves];
  __shared__ int slow;  // packed-tab fast path refused (workgroup-uniform after a barrier)
  __shared__ uint32_t whist[kWaves][64];  // copy_chunks' per-wave chunk histograms
  shf_tab_job* job = jobs + blockIdx.x;
  const uint32_t t = threadIdx.x, lane = t & 63u, wave = t >> 6;
  const uint64_t src_len = job->src_len;
  const bool moving = job->tab_new != SHF_TAB_NONE;
  const uint8_t* src = src_base + job->src;
  const uint16_t* map = moving ? maps + (uint64_t)job->map * 2048u : maps;
  const uint32_t len_len = prm.fixed ? 0u : 4u;  // shf.c:674
  const uint32_t factor = prm.data_needed_factor ? prm.data_needed_factor : 1u;
  const uint32_t tab_new = job->tab_new, keep_type = job->keep_type, move_type = job->move_type;
  const uint64_t cap = job->cap;
  if (t == 0) {
    max_len = 0;
    len_total = 0;
    // every byte a job names lies in its buffer; images are 8-B aligned
    bad = src_len < kTabData || job->src > src_bytes || src_len > src_bytes - job->src || cap < kTabData ||
          job->keep > dst_bytes || cap > dst_bytes - job->keep ||
          (moving && (job->move > dst_bytes || cap > dst_bytes - job->move || job->map >= n_maps)) ||
          ((job->src | job->keep | (moving ? job->move : 0)) & 7u) != 0;
  }
  __syncthreads();
  if (bad) {
    if (t == 0) flag(job, SHF_HB_ERR_ARG);
    return;
  }
  uint8_t* keep = dst_base + job->keep;
  uint8_t* move = moving ? dst_base + job->move : nullptr;
  const RecList LK{e_end, e_pos, 0, 1}, LM{e_end, e_pos, (int32_t)kTabRefs - 1, -1};
  const uint64_t d0k = reinterpret_cast<uintptr_t>(keep + kTabData), d0m = reinterpret_cast<uintptr_t>(move + kTabData);
  // what the segments before this one hold (workgroup-uniform)
  uint64_t done_keep = 0, done_move = 0;   // data bytes
  uint32_t refs_keep = 0, refs_move = 0;   // records
  uint64_t next_k = d0k >> 4, next_m = d0m >> 4;  // the first chunk not yet copied

  // Packed tabs (variable lengths, tab_data_free == 0: no deleted record, so
  // the records tile [data, tab_used) in insertion order, shf.c:601-609): a
  // record's length is the distance from its position to the next record's.
  // The positions are bucket-sorted in LDS (the record lists' arrays, free
  // until the segment loop), so no record's two length words are read (a
  // dependent pair of scattered reads per record). Anything unexpected
  // (positions outside the data, a shared position, a record under 9 B, a
  // crowded bucket) falls back to reading the length words.
  uint32_t lenreg[kSegs * kSlabs / 2];  // two u16 record lengths per word (longer records: no fast path)
  uint32_t mv_all = 0;                   // fast path, early move: bit seg * kSlabs + j = that ref moves
  bool fast = false;
  if (!prm.fixed) {
    const uint32_t tab_used = load_u32(src + 4), data_free = load_u32(src + 16);  // shf.private.h:59-65
    if (data_free == 0 && tab_used >= kTabData && tab_used <= src_len && tab_used - kTabData < (1u << 30)) {
      constexpr uint32_t kBuckets = 4096, kPer = kBuckets / kThreads;
      uint32_t* pos_by_ref = e_end;   // then each ref's record length
      uint32_t* counts = e_pos;       // bucket counts, then starts
      uint16_t* sorted = reinterpret_cast<uint16_t*>(e_pos + kBuckets);  // refs in position order
      const uint32_t w = (tab_used - kTabData) / kBuckets + 1u;  // bucket width in bytes
#pragma unroll
      for (uint32_t i = 0; i < kPer; ++i) counts[t * kPer + i] = 0;
      if (t == 0) slow = 0;
      seg_barrier();
      uint32_t pk[kSegs * kSlabs], slot[kSegs * kSlabs];
      uint32_t wk[kSegs * kSlabs];
#pragma unroll
      for (uint32_t k = 0; k < kSegs * kSlabs; ++k) {
        const uint32_t r = (k / kSlabs) * kSegRefs + (k % kSlabs) * kThreads + t;
        const uint2 ref = *reinterpret_cast<const uint2*>(src + kTabHdr + 8u * r);
        wk[k] = ref.x;
        pk[k] = ref.y;
      }
      // every ref's destination image now (shf.c:765-767), so the segment
      // loop's scans wait on no global read
      if (moving) {
#pragma unroll
        for (uint32_t k = 0; k < kSegs * kSlabs; ++k)
          mv_all |= (uint32_t)(pk[k] != 0 && map[wk[k] & 0x7ffu] == tab_new) << k;
      }
#pragma unroll
      for (uint32_t k = 0; k < kSegs * kSlabs; ++k) {
        const uint32_t r = (k / kSlabs) * kSegRefs + (k % kSlabs) * kThreads + t;
        slot[k] = 0;
        if (pk[k] == 0) continue;
        if (pk[k] < kTabData || pk[k] >= tab_used) {
          slow = 1;
          pk[k] = 0;
          continue;
        }
        pos_by_ref[r] = pk[k];
        slot[k] = atomicAdd(&counts[(pk[k] - kTabData) / w], 1u);
      }
      seg_barrier();
      // exclusive scan of the bucket counts (thread t: buckets [t * kPer, t * kPer + kPer))
      uint32_t c[kPer], sum = 0;
#pragma unroll
      for (uint32_t i = 0; i < kPer; ++i) {
        c[i] = counts[t * kPer + i];
        sum += c[i];
        if (c[i] > 64u) slow = 1;  // insertion sort below stays short
      }
      const uint32_t incl = wave_incl_scan(sum);
      if (lane == 63) wtot[wave] = incl;
      seg_barrier();
      uint32_t before = 0, n_used = 0;
#pragma unroll
      for (uint32_t v = 0; v < kWaves; ++v) {
        before += v < wave ? wtot[v] : 0u;
        n_used += wtot[v];
      }
      uint32_t at = before + incl - sum;
#pragma unroll
      for (uint32_t i = 0; i < kPer; ++i) {
        counts[t * kPer + i] = at;
        at += c[i];
      }
      seg_barrier();
#pragma unroll
      for (uint32_t k = 0; k < kSegs * kSlabs; ++k) {
        const uint32_t r = (k / kSlabs) * kSegRefs + (k % kSlabs) * kThreads + t;
        if (pk[k]) sorted[counts[(pk[k] - kTabData) / w] + slot[k]] = (uint16_t)r;
      }
      seg_barrier();
      if (!slow) {  // order each bucket by position (a few entries each)
#pragma unroll
        for (uint32_t i = 0; i < kPer; ++i) {
          const uint32_t b0 = counts[t * kPer + i];
          for (uint32_t x = 1; x < c[i]; ++x) {
            const uint16_t rx = sorted[b0 + x];
            const uint32_t px = pos_by_ref[rx];
            uint32_t y = x;
            while (y > 0 && pos_by_ref[sorted[b0 + y - 1]] > px) {
              sorted[b0 + y] = sorted[b0 + y - 1];
              --y;
            }
            sorted[b0 + y] = rx;
          }
        }
      }
      seg_barrier();
      uint32_t lens[kSegs * kSlabs];
      if (!slow) {
#pragma unroll
        for (uint32_t m = 0; m < kSegs * kSlabs; ++m) {
          const uint32_t i = t + m * kThreads;
          lens[m] = 0;
          if (i < n_used) {
            const uint32_t p0 = pos_by_ref[sorted[i]];
            const uint32_t nx = i + 1 < n_used ? pos_by_ref[sorted[i + 1]] : tab_used;
            lens[m] = nx - p0;
            if (lens[m] < 9u || lens[m] > 0xffffu || (i == 0 && p0 != kTabData)) slow = 1;
          }
        }
      }
      seg_barrier();
      fast = !slow;
      if (fast) {
#pragma unroll
        for (uint32_t m = 0; m < kSegs * kSlabs; ++m) {
          const uint32_t i = t + m * kThreads;
          if (i < n_used) pos_by_ref[sorted[i]] = lens[m];  // now each ref's record length
        }
      }
      seg_barrier();
      if (fast) {
#pragma unroll
        for (uint32_t k = 0; k < kSegs * kSlabs; k += 2) {
          const uint32_t r = (k / kSlabs) * kSegRefs + (k % kSlabs) * kThreads + t;
          const uint32_t r1 = ((k + 1) / kSlabs) * kSegRefs + ((k + 1) % kSlabs) * kThreads + t;
          lenreg[k / 2] = (pk[k] ? pos_by_ref[r] : 0u) | ((pk[k + 1] ? pos_by_ref[r1] : 0u) << 16);
        }
      }
      // (the segment loop's first barrier orders these reads before the lists reuse the arrays)
    }
  }

  for (uint32_t seg = 0; seg < kSegs; ++seg) {
    // 1. this thread's refs {tab:11 | rnd:21, pos} (shf.private.h:48-52) and their record lengths
    uint32_t w0[kSlabs], pos[kSlabs], len[kSlabs], kl[kSlabs];
    bool mine_bad = false;
    uint32_t lseg[kSlabs];  // this segment's lengths from positions (constant indices: registers, not scratch)
#pragma unroll
    for (uint32_t j = 0; j < kSlabs; ++j) {
      uint32_t v = lenreg[j / 2];
#pragma unroll
      for (uint32_t g = 1; g < kSegs; ++g) v = seg == g ? lenreg[(g * kSlabs + j) / 2] : v;
      lseg[j] = (j & 1u) ? v >> 16 : v & 0xffffu;
    }
#pragma unroll
    for (uint32_t j = 0; j < kSlabs; ++j) {
      const uint32_t r = seg * kSegRefs + j * kThreads + t;
      const uint2 ref = *reinterpret_cast<const uint2*>(src + kTabHdr + 8u * r);  // 8-B aligned
      w0[j] = ref.x;
      pos[j] = ref.y;
    }
    // SHF_TAB_REF_COPY's lengths (shf.c:636-637): the key length word, then the value length word after the key
#pragma unroll
    for (uint32_t j = 0; j < kSlabs; ++j) {
      kl[j] = prm.fixed_key_len;
      if (fast) continue;  // positions checked by the fast path's sort
      if (!prm.fixed && pos[j] != 0) {
        if (pos[j] < kTabData || (uint64_t)pos[j] + 9u > src_len) mine_bad = true;
        else if (!fast) kl[j] = load_u32(src + pos[j] + 1);
      }
    }
    uint32_t to_move = 0;  // bit j: ref of slab j goes to the move image
    if (fast) {  // lengths and images known; the refs just loaded are first needed by step 3
#pragma unroll
      for (uint32_t j = 0; j < kSlabs; ++j) len[j] = lseg[j];
      to_move = (mv_all >> (seg * kSlabs)) & ((1u << kSlabs) - 1u);
    } else
#pragma unroll
    for (uint32_t j = 0; j < kSlabs; ++j) {
      len[j] = 0;
      if (pos[j] == 0) continue;  // ref unused
      const uint64_t p = pos[j];
      uint32_t vl = prm.fixed_val_len;
      if (!prm.fixed) {
        if (p < kTabData || (!fast && p + 9u + kl[j] > src_len)) {
          mine_bad = true;
          continue;
        }
        if (!fast) vl = load_u32(src + p + 5 + kl[j]);
      }
      const uint64_t l = fast ? (uint64_t)lseg[j] : 1ull + len_len + kl[j] + len_len + vl;
      if (p < kTabData || p + l > src_len || l > 0xffffffffull) {
        mine_bad = true;
        continue;
      }
      len[j] = (uint32_t)l;
      to_move |= (uint32_t)(moving && map[w0[j] & 0x7ffu] == tab_new) << j;  // shf.c:765-767
    }
    if (mine_bad) bad = 1;
    {
      // the longest record, and the exact u64 total of the lengths: the u32 scans
      // below would wrap unnoticed on a corrupt image whose refs repeat one large
      // record (each within the image, their sum not)
      uint32_t m = 0;
      uint64_t sum = 0;
#pragma unroll
      for (uint32_t j = 0; j < kSlabs; ++j) {
        m = max(m, len[j]);
        sum += len[j];
      }
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) {
        m = max(m, (uint32_t)__shfl_xor((int)m, d));
        sum += (uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)sum, d) |
               ((uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)(sum >> 32), d) << 32);
      }
      if (lane == 0) {  // read after the segment loop's barriers
        atomicMax(&max_len, m);
        atomicAdd(&len_total, (unsigned long long)sum);
      }
    }

    // 2. scans in ref order (slab by slab, thread by thread): in the wave, then over the waves
    //    through LDS. Per ref: its size in keep, in move, and the keep and move record counts
    //    packed in one word. The in-wave scans are recomputed after the barrier rather than held.
#pragma unroll
    for (uint32_t j = 0; j < kSlabs; ++j) {
      const bool mv = (to_move >> j) & 1u;
      const uint32_t ik = wave_incl_scan(mv ? 0u : len[j]), im = wave_incl_scan(mv ? len[j] : 0u);
      const uint32_t ic = wave_incl_scan(len[j] ? (mv ? 0x10000u : 1u) : 0u);
      if (lane == 63) {
        wsum[seg & 1][j][0][wave] = ik;
        wsum[seg & 1][j][1][wave] = im;
        wsum[seg & 1][j][2][wave] = ic;
      }
    }
    seg_barrier();
    uint64_t seg_k = 0, seg_m = 0;  // this segment's keep and move bytes so far
    uint32_t seg_c = 0;             // and records (packed: keep low, move high half)
    // 3. each ref's record offset in its image, its list entry, its row entry in both images
#pragma unroll
    for (uint32_t j = 0; j < kSlabs; ++j) {
      const bool mv = (to_move >> j) & 1u, used = len[j] != 0;
      const uint32_t ik = wave_incl_scan(mv ? 0u : len[j]), im = wave_incl_scan(mv ? len[j] : 0u);
      const uint32_t ic = wave_incl_scan(used ? (mv ? 0x10000u : 1u) : 0u);
      uint32_t bk = 0, bm = 0, bc = 0, ak = 0, am = 0, ac = 0;  // before this wave / whole slab
#pragma unroll
      for (uint32_t w = 0; w < kWaves; ++w) {
        const uint32_t vk = wsum[seg & 1][j][0][w], vm = wsum[seg & 1][j][1][w], vc = wsum[seg & 1][j][2][w];
        ak += vk;
        am += vm;
        ac += vc;
        if (w < wave) {
          bk += vk;
          bm += vm;
          bc += vc;
        }
      }
      const uint32_t r = seg * kSegRefs + j * kThreads + t;
      const uint32_t end = mv ? (uint32_t)(done_move + seg_m) + bm + im : (uint32_t)(done_keep + seg_k) + bk + ik;
      const uint32_t at = kTabData + end - len[j];  // inclusive end - size = this record's offset
      if (used) {
        const uint32_t c = seg_c + bc + ic;  // inclusive counts in this segment
        const uint32_t rank = mv ? refs_move + (c >> 16) - 1u : refs_keep + (c & 0xffffu) - 1u;
        const uint32_t i = mv ? kTabRefs - 1u - rank : rank;
        e_end[i] = end;
        e_pos[i] = pos[j];
      }
      *reinterpret_cast<uint2*>(keep + kTabHdr + 8u * r) = (used && !mv) ? make_uint2(w0[j], at) : make_uint2(0u, 0u);
      if (moving)
        *reinterpret_cast<uint2*>(move + kTabHdr + 8u * r) = (used && mv) ? make_uint2(w0[j], at) : make_uint2(0u, 0u);
      seg_k += ak;
      seg_m += am;
      seg_c += ac;
    }
    const uint64_t seg_tot[4] = {seg_k, seg_m, seg_c & 0xffffu, seg_c >> 16};
    done_keep += seg_tot[0];
    done_move += seg_tot[1];
    refs_keep += (uint32_t)seg_tot[2];
    refs_move += (uint32_t)seg_tot[3];
    if (t == 0 && (kTabData + done_keep > cap || (moving && kTabData + done_move > cap) ||
                   kTabData + done_keep + done_move > 0xffffffffull || kTabData + len_total > 0xffffffffull))
      bad = 1;
    seg_barrier();
    if (bad) break;  // workgroup-uniform; nothing past cap was or will be written

    // 4. the data chunks this segment completes (every byte below done_*)
    const uint64_t end_k = (d0k + done_keep) >> 4, end_m = (d0m + done_move) >> 4;
    copy_chunks(src, src_len, LK, refs_keep, done_keep, d0k, next_k, end_k, keep_type, t, whist[wave]);
    next_k = end_k;
    if (moving) {
      copy_chunks(src, src_len, LM, refs_move, done_move, d0m, next_m, end_m, move_type, t, whist[wave]);
      next_m = end_m;
    }
  }
  if (bad) {
    if (t == 0) flag(job, SHF_HB_ERR_ARG);
    return;
  }
  // the last partial chunk of each image
  copy_chunks(src, src_len, LK, refs_keep, done_keep, d0k, next_k, (d0k + done_keep + 15u) >> 4, keep_type, t, whist[wave]);
  if (moving) copy_chunks(src, src_len, LM, refs_move, done_move, d0m, next_m, (d0m + done_move + 15u) >> 4, move_type, t, whist[wave]);

  // 5. headers: tab_size (replayed growth), tab_used, tab_refs_used (SHF_TAB_APPEND and
  //    SHF_TAB_REF_COPY both count each copied ref, shf.c:608, :651), free pos, free, data used
  if (wave == 0 || (moving && wave == 1)) {
    const bool m = wave == 1;
    // When no record needs more than a page (len x factor <= 4096), each growth
    // SHF_TAB_APPEND makes is exactly one page (tab sizes are page multiples),
    // so the size is the first page multiple that holds all the data: no replay.
    const uint64_t total_m = m ? done_move : done_keep;
    const uint64_t size = (uint64_t)max_len * factor <= kPage
                              ? max(mod_page(kTabData), mod_page(kTabData + total_m))
                              : replay_tab_size(m ? LM : LK, m ? refs_move : refs_keep, factor, lane);
    if (lane == 0) {
      uint8_t* img = m ? move : keep;
      const uint64_t total = m ? done_move : done_keep;
      store_u32(img + 0, (uint32_t)size);
      store_u32(img + 4, (uint32_t)(kTabData + total));
      store_u32(img + 8, 2u * (m ? refs_move : refs_keep));
      store_u32(img + 12, 0u);
      store_u32(img + 16, 0u);
      store_u32(img + 20, (uint32_t)total);
    }
  }
  if (t == 0) flag(job, SHF_HB_OK);
}


hipError_t launch_tab_split(const void* src, uint64_t src_bytes, void* dst, uint64_t dst_bytes, shf_tab_job* jobs,
                            uint32_t n_jobs, const uint16_t* maps, uint32_t n_maps, const shf_tab_params& prm,
                            hipStream_t st) {
  if (n_jobs == 0) return hipSuccess;
  hipLaunchKernelGGL(k_tab_split, dim3(n_jobs), dim3(kThreads), 0, st, reinterpret_cast<const uint8_t*>(src),
                     src_bytes, reinterpret_cast<uint8_t*>(dst), dst_bytes, jobs, maps, n_maps, prm);
  return hipGetLastError();
}

}  // namespace shfhb

