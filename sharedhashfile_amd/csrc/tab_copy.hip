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
// One 512-thread workgroup per tab (a job); thread t owns row t (16 refs,
// 128 B, read and written with 16-B accesses). Each thread reads its refs and
// their records' two length words, the workgroup scans the record sizes (keep
// and move separately: wave shuffles, then the 8 wave totals through LDS),
// each thread writes its row into both images and copies its records, 8 at a
// time piece by piece (16-B unaligned loads and stores, so a wave keeps up to
// 8 of its records' loads in flight per lane; a record's last partial piece is
// stored exactly), and two waves replay the two images' growth (SHF_TAB_APPEND's
// tab_size, :562-565) with a wave-wide forward search of the scanned ends.
// HBM-bound: each record is read once (plus its two length words) and written
// once, the 64-KiB rows are read once and written twice.
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
constexpr uint32_t kThreads = 512;
constexpr uint32_t kWaves = kThreads / 64;
constexpr uint32_t kRefsPerThread = kTabRefs / kThreads;  // 16: one row

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

// Wave-wide inclusive scan of a u32.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, uint32_t lane) {
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t u = (uint32_t)__shfl_up((int)v, d);
    if (lane >= d) v += u;
  }
  return v;
}

// tab_size after appending an image's records in order to a fresh tab
// (SHF_GET_TAB_MMAP's initial size MOD_PAGE(sizeof(SHF_TAB_MMAP)), then
// SHF_TAB_APPEND's growth MOD_PAGE(tab_size + data_needed * factor) whenever a
// record does not fit). ends[0..n) = data bytes up to and including each of
// the image's records (increasing). One wave; every lane returns the size.
// The first record whose end exceeds the room is found 64 ends at a time,
// moving forward only.
__device__ uint64_t replay_tab_size(const uint32_t* ends, uint32_t n, uint32_t factor, uint32_t lane) {
  uint64_t size = mod_page(kTabData);
  uint32_t i0 = 0;
  for (;;) {
    const uint64_t room = size - kTabData;
    uint64_t hit = 0;
    while (i0 < n) {
      hit = __ballot(i0 + lane < n && (uint64_t)ends[i0 + lane] > room);
      if (hit) break;
      i0 += 64;
    }
    if (!hit) return size;
    i0 += (uint32_t)__builtin_ctzll(hit);  // first record that does not fit
    const uint32_t len = ends[i0] - (i0 ? ends[i0 - 1] : 0u);
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

__device__ __forceinline__ unsigned __int128 low_bytes128(uint32_t n) {  // n in [0, 16]
  return n >= 16u ? ~(unsigned __int128)0 : (((unsigned __int128)1 << (8 * n)) - 1);
}

__device__ __forceinline__ void flag(shf_tab_job* job, int v) {
  *reinterpret_cast<volatile int32_t*>(&job->status) = v;
}

}  // namespace

__global__ __launch_bounds__(kThreads) void k_tab_split(const uint8_t* __restrict__ src_base, uint64_t src_bytes,
                                                        uint8_t* dst_base, uint64_t dst_bytes, shf_tab_job* jobs,
                                                        const uint16_t* __restrict__ maps, uint32_t n_maps,
                                                        shf_tab_params prm) {
  // the records of both images in image order: keep's at [0, refs_keep), move's after them;
  // e_end = the record's end in its image's data (inclusive scan of the sizes), e_pos = its source byte
  __shared__ uint32_t e_end[kTabRefs];
  __shared__ uint32_t e_pos[kTabRefs];
  __shared__ uint32_t wsum[4][kWaves];     // per wave: keep bytes, move bytes, keep refs, move refs
  __shared__ int bad;
  shf_tab_job* job = jobs + blockIdx.x;
  const uint32_t t = threadIdx.x, lane = t & 63u, wave = t >> 6;
  const uint64_t src_len = job->src_len;
  const bool moving = job->tab_new != SHF_TAB_NONE;
  const uint8_t* src = src_base + job->src;
  const uint16_t* map = moving ? maps + (uint64_t)job->map * 2048u : maps;
  const uint32_t len_len = prm.fixed ? 0u : 4u;  // shf.c:674
  const uint32_t factor = prm.data_needed_factor ? prm.data_needed_factor : 1u;
  if (t == 0) {
    // every byte a job names lies in its buffer; images are 8-B aligned
    const uint64_t cap = job->cap;
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

  // 1. this thread's row: refs {tab:11 | rnd:21, pos} (shf.private.h:48-52), record lengths
  uint32_t w0[kRefsPerThread], pos[kRefsPerThread], len[kRefsPerThread];
  const u32x4* row = reinterpret_cast<const u32x4*>(src + kTabHdr + (uint64_t)t * kRefsPerThread * 8u);
#pragma unroll
  for (uint32_t q = 0; q < kRefsPerThread / 2; ++q) {  // 8-B aligned: two 8-B loads' worth as one 16-B load
    const u32x4 r = *reinterpret_cast<const u32x4_a1*>(row + q);
    w0[2 * q] = r.x;
    pos[2 * q] = r.y;
    w0[2 * q + 1] = r.z;
    pos[2 * q + 1] = r.w;
  }
  // SHF_TAB_REF_COPY's lengths (shf.c:636-637): the key length word, then the value length word after the key
  bool mine_bad = false;
  uint32_t kl[kRefsPerThread];
#pragma unroll
  for (uint32_t j = 0; j < kRefsPerThread; ++j) {
    kl[j] = prm.fixed_key_len;
    if (!prm.fixed && pos[j] != 0) {
      if (pos[j] < kTabData || (uint64_t)pos[j] + 9u > src_len) mine_bad = true;
      else kl[j] = load_u32(src + pos[j] + 1);
    }
  }
  uint32_t to_move = 0;  // bit j: ref j goes to the move image
  uint32_t sum_keep = 0, sum_move = 0, n_keep = 0, n_move = 0;
#pragma unroll
  for (uint32_t j = 0; j < kRefsPerThread; ++j) {
    len[j] = 0;
    if (pos[j] == 0) continue;  // ref unused
    const uint64_t p = pos[j];
    uint32_t vl = prm.fixed_val_len;
    if (!prm.fixed) {
      if (p < kTabData || p + 9u + kl[j] > src_len) {
        mine_bad = true;
        continue;
      }
      vl = load_u32(src + p + 5 + kl[j]);
    }
    const uint64_t l = 1ull + len_len + kl[j] + len_len + vl;
    if (p < kTabData || p + l > src_len || l > 0xffffffffull) {
      mine_bad = true;
      continue;
    }
    len[j] = (uint32_t)l;
    const bool mv = moving && map[w0[j] & 0x7ffu] == job->tab_new;  // shf.c:765-767
    to_move |= (uint32_t)mv << j;
    if (mv) {
      sum_move += (uint32_t)l;
      ++n_move;
    } else {
      sum_keep += (uint32_t)l;
      ++n_keep;
    }
  }
  if (mine_bad) bad = 1;

  // 2. exclusive scans of the per-thread sums: in the wave, then over the waves
  const uint32_t ik = wave_incl_scan(sum_keep, lane), im = wave_incl_scan(sum_move, lane);
  const uint32_t ck = wave_incl_scan(n_keep, lane), cm = wave_incl_scan(n_move, lane);
  if (lane == 63) {
    wsum[0][wave] = ik;
    wsum[1][wave] = im;
    wsum[2][wave] = ck;
    wsum[3][wave] = cm;
  }
  __syncthreads();
  uint64_t total_keep = 0, total_move = 0;
  uint32_t base_keep = 0, base_move = 0, refs_keep = 0, refs_move = 0;
#pragma unroll
  for (uint32_t w = 0; w < kWaves; ++w) {
    total_keep += wsum[0][w];
    total_move += wsum[1][w];
    refs_keep += wsum[2][w];
    refs_move += wsum[3][w];
    if (w < wave) {
      base_keep += wsum[0][w];
      base_move += wsum[1][w];
    }
  }
  if (t == 0 && (kTabData + total_keep > job->cap || (moving && kTabData + total_move > job->cap) ||
                 kTabData + total_keep + total_move > 0xffffffffull))
    bad = 1;
  uint32_t rank_keep = ck - n_keep, rank_move = refs_keep + cm - n_move;  // this thread's first record ranks
#pragma unroll
  for (uint32_t w = 0; w < kWaves; ++w)
    if (w < wave) {
      rank_keep += wsum[2][w];
      rank_move += wsum[3][w];
    }
  uint32_t run_keep = base_keep + ik - sum_keep, run_move = base_move + im - sum_move;  // exclusive
  uint32_t at[kRefsPerThread];  // each ref's record offset in its image
#pragma unroll
  for (uint32_t j = 0; j < kRefsPerThread; ++j) {
    const bool mv = (to_move >> j) & 1u;
    at[j] = kTabData + (mv ? run_move : run_keep);
    if (len[j]) {
      const uint32_t r = mv ? rank_move++ : rank_keep++;
      e_end[r] = (mv ? run_move : run_keep) + len[j];
      e_pos[r] = pos[j];
    }
    run_keep += mv ? 0u : len[j];
    run_move += mv ? len[j] : 0u;
  }
  __syncthreads();
  if (bad) {
    if (t == 0) flag(job, SHF_HB_ERR_ARG);
    return;
  }

  // 3. this row in both images (a ref not copied to an image is 0 there: fresh tabs)
  uint8_t* keep = dst_base + job->keep;
  uint8_t* move = moving ? dst_base + job->move : nullptr;
  u32x4* krow = reinterpret_cast<u32x4*>(keep + kTabHdr + (uint64_t)t * kRefsPerThread * 8u);
  u32x4* mrow = moving ? reinterpret_cast<u32x4*>(move + kTabHdr + (uint64_t)t * kRefsPerThread * 8u) : nullptr;
#pragma unroll
  for (uint32_t q = 0; q < kRefsPerThread / 2; ++q) {
    u32x4 k = {0u, 0u, 0u, 0u}, m = {0u, 0u, 0u, 0u};
#pragma unroll
    for (uint32_t h = 0; h < 2; ++h) {
      const uint32_t j = 2 * q + h;
      const bool used = len[j] != 0, mv = (to_move >> j) & 1u;
      const uint32_t a = (used && !mv) ? w0[j] : 0u, b = (used && !mv) ? at[j] : 0u;
      const uint32_t c = (used && mv) ? w0[j] : 0u, d = (used && mv) ? at[j] : 0u;
      if (h == 0) {
        k.x = a, k.y = b, m.x = c, m.y = d;
      } else {
        k.z = a, k.w = b, m.z = c, m.w = d;
      }
    }
    *reinterpret_cast<u32x4_a1*>(krow + q) = k;  // 8-B aligned images
    if (moving) *reinterpret_cast<u32x4_a1*>(mrow + q) = m;
  }

  // 4. the records: each image's data region as 16-B destination chunks
  //    (absolute 16-B alignment), consecutive chunks on consecutive lanes, four
  //    per lane in flight. A chunk's bytes come from the record holding its first
  //    byte (binary search of the ends) and, where it crosses record ends, the
  //    next ones; each record's first byte is its SHF_DATA_TYPE, written as the
  //    job says (shf.c:593-596). Only the images' data bytes are written.
#ifndef SHFHB_TAB_CHUNKS
#define SHFHB_TAB_CHUNKS 4
#endif
  constexpr uint32_t kChunksPerLane = SHFHB_TAB_CHUNKS;
#pragma unroll 1
  for (uint32_t m = 0; m < (moving ? 2u : 1u); ++m) {
    const uint32_t b0 = m ? refs_keep : 0u, nrec = m ? refs_move : refs_keep;
    const uint64_t total = m ? total_move : total_keep;
    if (total == 0) continue;
    const uint32_t type = m ? job->move_type : job->keep_type;
    const uint64_t d0 = reinterpret_cast<uintptr_t>((m ? move : keep) + kTabData);  // absolute
    const uint64_t c0 = d0 >> 4, nchunks = ((d0 + total + 15u) >> 4) - c0;
    for (uint64_t base = 0; base < nchunks; base += kChunksPerLane * kThreads) {
      unsigned __int128 v[kChunksPerLane];
      uint32_t k[kChunksPerLane], lo[kChunksPerLane], hi[kChunksPerLane], st[kChunksPerLane];
      int64_t a[kChunksPerLane];
#pragma unroll
      for (uint32_t q = 0; q < kChunksPerLane; ++q) {
        const uint64_t i = base + q * kThreads + t;
        a[q] = (int64_t)((c0 + i) << 4) - (int64_t)d0;  // the chunk's first byte in the image's data
        lo[q] = a[q] < 0 ? 0u : (uint32_t)a[q];
        hi[q] = (uint32_t)min<int64_t>(a[q] + 16, (int64_t)total);
        if (i >= nchunks) hi[q] = lo[q];
        uint32_t l = 0, h = nrec;  // first record ending past lo
        while (l < h) {
          const uint32_t mid = (l + h) >> 1;
          if (e_end[b0 + mid] > lo[q]) h = mid;
          else l = mid + 1;
        }
        k[q] = b0 + l;
        if (lo[q] < hi[q]) {
          st[q] = k[q] > b0 ? e_end[k[q] - 1] : 0u;
          v[q] = load16(src, src_len, (uint64_t)e_pos[k[q]] + (lo[q] - st[q]));
        }
      }
#pragma unroll
      for (uint32_t q = 0; q < kChunksPerLane; ++q) {
        if (lo[q] >= hi[q]) continue;
        unsigned __int128 out = 0, x = v[q];
        uint32_t b = lo[q], s0 = st[q], kk = k[q];
        for (;;) {
          const uint32_t e = e_end[kk], take = min(e, hi[q]) - b, o = (uint32_t)(b - a[q]);
          if (b == s0) x = (x & ~(unsigned __int128)0xff) | type;
          out |= (x & low_bytes128(take)) << (8 * o);
          b += take;
          if (b >= hi[q]) break;
          s0 = e;
          ++kk;
          x = load16(src, src_len, e_pos[kk]);
        }
        uint8_t* dst = reinterpret_cast<uint8_t*>((c0 + base + q * kThreads + t) << 4);
        const uint32_t o = (uint32_t)((int64_t)lo[q] - a[q]);  // the chunk's first byte it writes
        const uint32_t n = hi[q] - lo[q];
        if (n == 16u) {
          *reinterpret_cast<u32x4*>(dst) = u32x4{(uint32_t)out, (uint32_t)(out >> 32), (uint32_t)(out >> 64),
                                                 (uint32_t)(out >> 96)};
        } else {
          const unsigned __int128 y = out >> (8 * o);
          store_partial(dst + o, u32x4{(uint32_t)y, (uint32_t)(y >> 32), (uint32_t)(y >> 64), (uint32_t)(y >> 96)}, n);
        }
      }
    }
  }

  // 5. headers: tab_size (replayed growth), tab_used, tab_refs_used (SHF_TAB_APPEND and
  //    SHF_TAB_REF_COPY both count each copied ref, shf.c:608, :651), free pos, free, data used
  if (wave == 0 || (moving && wave == 1)) {
    const bool m = wave == 1;
    const uint64_t size = replay_tab_size(e_end + (m ? refs_keep : 0u), m ? refs_move : refs_keep, factor, lane);
    if (lane == 0) {
      uint8_t* img = m ? move : keep;
      const uint64_t total = m ? total_move : total_keep;
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
