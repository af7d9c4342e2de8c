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
// One 256-thread workgroup per tab (a job). Thread t owns refs [32t, 32t+32)
// (rows 2t and 2t+1): it reads their refs and record lengths, the workgroup
// scans the lengths (keep and move separately) into LDS, then each thread
// writes its refs into both images' rows and copies its records; one lane per
// image replays the tab's growth (SHF_TAB_APPEND's tab_size, :562-565) by
// binary search over the scanned ends. HBM-bound: every data byte is read once
// and written once, the 64-KiB rows are read once and written twice.
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
constexpr uint32_t kThreads = 256;
constexpr uint32_t kRefsPerThread = kTabRefs / kThreads;  // 32

__device__ __forceinline__ uint64_t mod_page(uint64_t b) { return ((b - 1) / kPage + 1) * kPage; }  // shf.defines.h:76

// Unaligned little-endian u32 of global memory (records start at any byte).
__device__ __forceinline__ uint32_t load_u32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

__device__ __forceinline__ void store_u32(uint8_t* p, uint32_t v) {
  p[0] = (uint8_t)v;
  p[1] = (uint8_t)(v >> 8);
  p[2] = (uint8_t)(v >> 16);
  p[3] = (uint8_t)(v >> 24);
}

// Copy len bytes, any alignment of either side: byte-wise up to a 4-aligned
// destination, then dwords assembled from the source (unaligned dword loads
// are legal on gfx950), then the tail bytes.
__device__ __forceinline__ void copy_bytes(uint8_t* dst, const uint8_t* src, uint32_t len) {
  uint32_t i = 0;
  while (i < len && ((reinterpret_cast<uintptr_t>(dst) + i) & 3u)) {
    dst[i] = src[i];
    ++i;
  }
  typedef uint32_t u32_a1 __attribute__((aligned(1)));
  for (; i + 4 <= len; i += 4)
    *reinterpret_cast<uint32_t*>(dst + i) = *reinterpret_cast<const u32_a1*>(src + i);
  for (; i < len; ++i) dst[i] = src[i];
}

// First index i of ends[0..n) (non-decreasing) with ends[i] > x, or n.
__device__ __forceinline__ uint32_t first_above(const uint32_t* ends, uint32_t n, uint64_t x) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if ((uint64_t)ends[mid] > x) hi = mid;
    else lo = mid + 1;
  }
  return lo;
}

// tab_size after appending the image's records in order to a fresh tab
// (SHF_GET_TAB_MMAP's initial size MOD_PAGE(sizeof(SHF_TAB_MMAP)), then
// SHF_TAB_APPEND's growth MOD_PAGE(tab_size + data_needed * factor) whenever a
// record does not fit). ends[i] = data bytes up to and including ref i.
__device__ uint64_t replay_tab_size(const uint32_t* ends, uint32_t factor) {
  uint64_t size = mod_page(kTabData);
  for (;;) {
    const uint32_t i = first_above(ends, kTabRefs, size - kTabData);  // first record that does not fit
    if (i == kTabRefs) return size;
    const uint32_t len = ends[i] - (i ? ends[i - 1] : 0u);
    size = mod_page(size + (uint64_t)len * factor);
  }
}

__device__ __forceinline__ void flag(shf_tab_job* job, int v) {
  *reinterpret_cast<volatile int32_t*>(&job->status) = v;
}

}  // namespace

__global__ __launch_bounds__(kThreads) void k_tab_split(const uint8_t* __restrict__ src_base, uint64_t src_bytes,
                                                        uint8_t* dst_base, uint64_t dst_bytes, shf_tab_job* jobs,
                                                        const uint16_t* __restrict__ maps, uint32_t n_maps,
                                                        shf_tab_params prm) {
  __shared__ uint32_t keep_end[kTabRefs];  // inclusive scans of the record sizes per image
  __shared__ uint32_t move_end[kTabRefs];
  __shared__ uint32_t part_keep[kThreads], part_move[kThreads];
  __shared__ int bad;
  shf_tab_job* job = jobs + blockIdx.x;
  const uint32_t t = threadIdx.x;
  const uint64_t src_len = job->src_len;
  const bool moving = job->tab_new != SHF_TAB_NONE;
  const uint8_t* src = src_base + job->src;
  const uint16_t* map = moving ? maps + (uint64_t)job->map * 2048u : maps;
  const uint32_t len_len = prm.fixed ? 0u : 4u;  // shf.c:674
  const uint32_t factor = prm.data_needed_factor ? prm.data_needed_factor : 1u;
  if (t == 0) {
    // every byte a job names lies in its buffer; images are 8-B aligned (refs are read and written as u64)
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

  // 1. this thread's refs: {tab:11 | rnd:21, pos} (shf.private.h:48-52), record lengths, destination
  uint32_t w0[kRefsPerThread], pos[kRefsPerThread], len[kRefsPerThread];
  uint32_t to_move = 0;  // bit j: ref j goes to the move image
  uint32_t sum_keep = 0, sum_move = 0;
  bool mine_bad = false;
  const uint8_t* rows = src + kTabHdr + (uint64_t)t * kRefsPerThread * 8u;
#pragma unroll
  for (uint32_t j = 0; j < kRefsPerThread; ++j) {
    const uint2 r = *reinterpret_cast<const uint2*>(rows + 8u * j);  // 8-B aligned in a tab image
    w0[j] = r.x;
    pos[j] = r.y;
    len[j] = 0;
    if (r.y == 0) continue;  // ref unused
    const uint64_t p = r.y;
    // SHF_TAB_REF_COPY's lengths (shf.c:636-637)
    uint32_t kl = prm.fixed_key_len, vl = prm.fixed_val_len;
    if (!prm.fixed) {
      if (p < kTabData || p + 5u > src_len) {
        mine_bad = true;
        continue;
      }
      kl = load_u32(src + p + 1);
      if (p + 1u + 4u + kl + 4u > src_len) {
        mine_bad = true;
        continue;
      }
      vl = load_u32(src + p + 1 + 4 + kl);
    }
    const uint64_t l = 1ull + len_len + kl + len_len + vl;
    if (p < kTabData || p + l > src_len || l > 0xffffffffull) {
      mine_bad = true;
      continue;
    }
    len[j] = (uint32_t)l;
    const bool mv = moving && map[r.x & 0x7ffu] == job->tab_new;  // shf.c:765-767
    to_move |= (uint32_t)mv << j;
    if (mv) sum_move += (uint32_t)l;
    else sum_keep += (uint32_t)l;
  }
  if (mine_bad) bad = 1;

  // 2. exclusive scan of the per-thread sums (Hillis-Steele over 256 entries)
  part_keep[t] = sum_keep;
  part_move[t] = sum_move;
  __syncthreads();
  for (uint32_t d = 1; d < kThreads; d <<= 1) {
    const uint32_t ak = t >= d ? part_keep[t - d] : 0u, am = t >= d ? part_move[t - d] : 0u;
    __syncthreads();
    part_keep[t] += ak;
    part_move[t] += am;
    __syncthreads();
  }
  const uint64_t total_keep = part_keep[kThreads - 1], total_move = part_move[kThreads - 1];
  uint32_t run_keep = part_keep[t] - sum_keep, run_move = part_move[t] - sum_move;  // exclusive
  if (t == 0 && (kTabData + total_keep > job->cap || (moving && kTabData + total_move > job->cap) ||
                 kTabData + total_keep + total_move > 0xffffffffull))
    bad = 1;
#pragma unroll
  for (uint32_t j = 0; j < kRefsPerThread; ++j) {
    const bool mv = (to_move >> j) & 1u;
    run_keep += mv ? 0u : len[j];
    run_move += mv ? len[j] : 0u;
    keep_end[t * kRefsPerThread + j] = run_keep;
    move_end[t * kRefsPerThread + j] = run_move;
  }
  __syncthreads();
  if (bad) {
    if (t == 0) flag(job, SHF_HB_ERR_ARG);
    return;
  }

  // 3. rows of both images (a ref not copied to an image is 0 there: fresh tabs), then the records
  uint8_t* keep = dst_base + job->keep;
  uint8_t* move = moving ? dst_base + job->move : nullptr;
#pragma unroll
  for (uint32_t j = 0; j < kRefsPerThread; ++j) {
    const uint32_t i = t * kRefsPerThread + j;
    const bool mv = (to_move >> j) & 1u;
    const bool used = len[j] != 0;
    const uint32_t at_keep = kTabData + keep_end[i] - (used && !mv ? len[j] : 0u);
    const uint32_t at_move = kTabData + move_end[i] - (used && mv ? len[j] : 0u);
    *reinterpret_cast<uint2*>(keep + kTabHdr + 8u * i) =
        (used && !mv) ? make_uint2(w0[j], at_keep) : make_uint2(0u, 0u);
    if (moving)
      *reinterpret_cast<uint2*>(move + kTabHdr + 8u * i) = (used && mv) ? make_uint2(w0[j], at_move) : make_uint2(0u, 0u);
    if (!used) continue;
    uint8_t* d = mv ? move + at_move : keep + at_keep;
    copy_bytes(d, src + pos[j], len[j]);
    d[0] = mv ? job->move_type : job->keep_type;  // the record's SHF_DATA_TYPE (shf.c:593-596)
  }

  // 4. headers: tab_size (replayed growth), tab_used, tab_refs_used (SHF_TAB_APPEND and
  //    SHF_TAB_REF_COPY both count each copied ref, shf.c:608, :651), free pos, free, data used
  if (t == 0 || (moving && t == 64)) {
    const bool m = t == 64;
    const uint32_t* ends = m ? move_end : keep_end;
    uint8_t* img = m ? move : keep;
    const uint64_t total = m ? total_move : total_keep;
    uint32_t n = 0;
    for (uint32_t i = 0, prev = 0; i < kTabRefs; ++i) {  // records = strictly increasing steps of the scan
      n += ends[i] != prev;
      prev = ends[i];
    }
    store_u32(img + 0, (uint32_t)replay_tab_size(ends, factor));
    store_u32(img + 4, (uint32_t)(kTabData + total));
    store_u32(img + 8, 2u * n);
    store_u32(img + 12, 0u);
    store_u32(img + 16, 0u);
    store_u32(img + 20, (uint32_t)total);
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
