// Internal launcher interface between the C-ABI layer (shf_hash_batch.hip) and
// the kernels (kernels.hip). Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/shf_hash_batch.h"

namespace shfhb {

// kOutHash: 16-B SHF_HASH records; kOutUid: 8-B packed UID parts;
// kOutProbe: 16-B shf_probe records (row pre-probe), plus the
// hashes when Sink::hash_out is set; kOutHashWin: the 16-B records plus each
// key's window byte (h1 & 0xff, shf.c:800) for the window order (win_order.hip);
// kOutUidWin: the 8-B UID parts plus the window byte.
enum OutMode { kOutHash = 0, kOutUid = 1, kOutProbe = 2, kOutHashWin = 3, kOutUidWin = 4 };
enum KernelChoice {
  kKernelAuto = 0,
  kKernelFixed16 = 1,
  kKernelTiled = 2,
  kKernelGeneric = 3,
  kKernelSpan = 4,
  kKernelRound = 5,
  kKernelSpanPP = 6
};

// Where a kernel's per-key result goes (passed by value as a kernel argument).
struct Sink {
  void* out = nullptr;                // n records of the OutMode's type
  void* hash_out = nullptr;           // kOutProbe: optional n x 16-B hashes
  const uint32_t* tab_slot = nullptr;  // kOutProbe: row index, see shf_hash_batch.h
  const uint8_t* rows = nullptr;
  uint64_t n_slots = 0;
  const uint8_t* map8 = nullptr;       // kOutProbe: compact copy of tab_slot (launch_compact_map), or null
  const uint32_t* win_tab = nullptr;
  uint32_t* status = nullptr;  // variable-length keys: set to 1 when a key's offsets are invalid
  uint8_t* wins = nullptr;     // kOutHashWin / kOutUidWin: n window bytes (rounded up to whole kWoChunk chunks)
  uint32_t* win_counts = nullptr;  // kOutHashWin, fused 16-B kernel: each chunk's 256 window counts
  uint16_t* win_sorted = nullptr;  // kOutHashWin, fused 16-B kernel: each chunk's order by window (win_rank.h)
};

// Window-order geometry, shared by the hashing kernels' fused epilogue and the
// order passes (win_order.hip): the batch is cut into chunks of kWoChunk keys;
// each chunk has one row of kWoBins counts.
constexpr uint32_t kWoChunk = 4096;
constexpr uint32_t kWoBins = 256;  // SHF_WINS_PER_SHF
// Counts are bin-major: bin b's row holds its count in chunk 0, 1, ... (the
// scan turns it into the exclusive prefix, entry [chunks] = the bin's total),
// rows kept 256-B aligned.
__host__ __device__ inline uint64_t wo_row_stride(uint64_t chunks) { return (chunks + 1 + 63) & ~63ull; }
// Workgroup g's chunk when the chunks are dealt XCD by XCD (workgroup g runs on
// XCD g % 8): the workgroups of one XCD take consecutive chunks, so each 128-B
// line of a counts row (32 consecutive chunks) is written through one L2.
__device__ inline uint32_t xcd_major(uint32_t g, uint32_t groups) {
  const uint32_t q = groups / 8u, r = groups % 8u, x = g % 8u;
  return x * q + min(x, r) + g / 8u;
}

// keys: device pointer to n * key_len bytes.
hipError_t launch_fixed(const void* keys, uint32_t key_len, uint64_t n, uint32_t seed, const Sink& sink,
                        int out_mode, hipStream_t st, int kernel);

// Key i = bytes[offsets[i] - off_base, offsets[i+1] - off_base); offsets on device.
// key_bytes: offsets[n] - offsets[0] when the caller knows it (sizes the span
// kernel's LDS window; 0 = unknown). It never changes results.
hipError_t launch_var(const void* bytes, const uint64_t* offsets, uint64_t off_base, uint64_t n, uint32_t seed,
                      const Sink& sink, int out_mode, hipStream_t st, int kernel = kKernelAuto,
                      uint64_t key_bytes = 0);

// *taken = atomic exchange of *word with 0 (one thread).
hipError_t launch_status_take(uint32_t* word, uint32_t* taken, hipStream_t st);

// Row pre-probe of precomputed hashes (n x 16 B on device) into sink.out.
hipError_t launch_probe_hashes(const void* hashes, uint64_t n, const Sink& sink, hipStream_t st);

// Compact copy of a row index's tab_slot map for the probes: map8[(win << 11) | tab2]
// = the entry's rank among its window's distinct indexed entries (0..253), 254 = not
// indexed (SHF_PROBE_NONE or a slot >= n_slots), 255 = a window with more than 254
// distinct entries (read tab_slot itself); win_tab[(win << 8) | rank] = the entry.
constexpr uint32_t kMapRanks = 254, kMapNone = 254, kMapEscape = 255;
hipError_t launch_compact_map(const uint32_t* tab_slot, uint64_t n_slots, uint8_t* map8, uint32_t* win_tab,
                              hipStream_t st);

// Tab part / shrink copy (tab_copy.hip): one workgroup per job, every pointer on device.
hipError_t launch_tab_split(const void* src, uint64_t src_bytes, void* dst, uint64_t dst_bytes, shf_tab_job* jobs,
                            uint32_t n_jobs, const uint16_t* maps, uint32_t n_maps, const shf_tab_params& prm,
                            hipStream_t st);

// Window order (win_order.hip): perm = the batch's key indices stably sorted by
// h1 & 0xff of their 16-B hash records; win_start (257 entries, optional) = the
// first position of each window in perm, then n. workspace: win_order_workspace_bytes(n).
uint64_t win_order_workspace_bytes(uint64_t n);
hipError_t launch_win_order(const void* hashes, uint64_t n, uint32_t* perm, uint32_t* win_start, void* workspace,
                            hipStream_t st);
// The workspace's window bytes, counts rows and chunk orders, for a hashing
// launch with kOutHashWin to fill; then launch_win_order_bytes orders from them
// (ranking the chunks' window bytes itself unless the hashing kernel ranked
// them: ranked).
uint8_t* win_order_wins(void* workspace, uint64_t n);
uint32_t* win_order_counts(void* workspace);
uint16_t* win_order_sorted(void* workspace, uint64_t n);
hipError_t launch_win_order_bytes(uint64_t n, bool ranked, uint32_t* perm, uint32_t* win_start, void* workspace,
                                  hipStream_t st);
// Fixed-length hash + window bytes (kOutHashWin): 16-B keys go through the fused
// kernel, which ranks each chunk itself (win_counts, win_sorted; *ranked = true).
hipError_t launch_fixed_win(const void* keys, uint32_t key_len, uint64_t n, uint32_t seed, const Sink& sink,
                            hipStream_t st, int kernel, bool* ranked);

}  // namespace shfhb
