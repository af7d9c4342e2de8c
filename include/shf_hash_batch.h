/*
 * shf_hash_batch.h -- C ABI of the MI355X batch key-hashing stage for
 * SharedHashFile.
 *
 * What it replaces. SharedHashFile hashes one key per call:
 *
 *     extern void shf_make_hash(const char *key, uint32_t key_len);
 *                                         -- /root/reference/src/shf.h:381
 *     -> MurmurHash3_x64_128(key, key_len, 12345, &shf_hash.u64[0])
 *                                         -- /root/reference/src/shf.c:456,
 *                                            /root/reference/src/murmurhash3.c:75
 *     result in the thread-local SHF_HASH shf_hash (u64[0] = h1, u64[1] = h2)
 *                                         -- /root/reference/src/shf.private.h:180-189
 *
 * The functions below compute the same 16 bytes for a whole batch of keys on
 * the GPU, bit-exact, and write them as an array of SHF_HASH-layout records
 * (struct shf_hash128). The results re-enter the unchanged put/get/del flow
 * through the reference's caller-supplied-hash seam: set shf_hash,
 * shf_hash_key and shf_hash_key_len per key and call shf_put_key_val() /
 * shf_get_key_val_copy() / shf_del_key_val() (as
 * /root/reference/src/test.9.shf.c:176-182 does). INTEGRATION.md shows the
 * helper a maintainer adds for that.
 *
 * Conventions.
 *   - Plain pointers and sizes only; no HIP or C++ types cross this ABI
 *     (streams are passed as `void *` holding a hipStream_t).
 *   - Every function returns SHF_HB_OK (0) or a negative SHF_HB_ERR_* code;
 *     nothing aborts. shf_hash_batch_strerror() names a code.
 *   - There is no CPU fallback: without a usable gfx950 device every hashing
 *     call returns SHF_HB_ERR_NODEV (or SHF_HB_ERR_ARCH).
 *   - Thread-safe. Host-memory calls stage through one pool of slots per
 *     device shared by every thread of the process (SHF_HB_POOL_MB, default
 *     64 MiB of device and 64 MiB of pinned memory per device, whatever the
 *     number of threads; slots of SHF_HB_STAGE_MB, default 16 MiB); a call
 *     borrows 1..SHF_HB_SLOTS (default 4) of them and waits only while every
 *     slot is on loan. Each thread holds one HIP stream and a few status
 *     words per device; when it exits they are kept for the next thread
 *     (no HIP call runs at thread exit), and shf_hash_batch_release() frees
 *     them. Device selection follows the calling
 *     thread's current HIP device (hipSetDevice), as HIP itself does.
 *   - Key lengths follow the reference's `const int len` parameter
 *     (murmurhash3.c:75): key_len and every variable key length must be
 *     < 2^31, else SHF_HB_ERR_ARG. A variable-length key is invalid when its
 *     offsets decrease (offsets[i+1] < offsets[i]) or span 2^31 bytes or more.
 *     Host-memory calls check the offsets before any transfer. Device-resident
 *     offsets are checked by the kernels: an invalid key's bytes are never
 *     read and its output record is left unwritten (every valid key of the
 *     batch is still hashed); the synchronous calls then return
 *     SHF_HB_ERR_ARG, and the asynchronous ones report it through
 *     shf_hash_batch_status().
 *   - fork. The HIP runtime's state (devices, streams, page-locked memory) and
 *     this library's staging pools and copy threads do not survive fork(). In
 *     a child forked after its parent made any call below that can reach HIP,
 *     every such call returns SHF_HB_ERR_FORKED at once, before any HIP call
 *     (it never hangs and never touches the parent's runtime state); exec()
 *     or a fresh process starts afresh. A child forked before the parent's
 *     first call uses the library normally. The reference's load test forks
 *     its workers (/root/reference/src/test.f.shf.c:274-336): fork them first,
 *     then hash in each. Calls exempt (no HIP):
 *     shf_win_order_workspace_bytes, shf_tab_part_redirect,
 *     shf_hash_batch_last_hip_error, _strerror, _version.
 */
#ifndef SHF_HASH_BATCH_H
#define SHF_HASH_BATCH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#if defined(__GNUC__)
#define SHF_HB_API __attribute__((visibility("default")))
#else
#define SHF_HB_API
#endif

/* Seed shf_make_hash() uses (/root/reference/src/shf.c:456). */
#define SHF_HASH_BATCH_SEED 12345u

/* Status codes. */
#define SHF_HB_OK 0
#define SHF_HB_ERR_ARG (-1)    /* bad argument: NULL buffer with n > 0, key length >= 2^31, bad mem kind */
#define SHF_HB_ERR_NODEV (-2)  /* no HIP device / runtime available */
#define SHF_HB_ERR_HIP (-3)    /* a HIP call failed; shf_hash_batch_last_hip_error() has the hipError_t */
#define SHF_HB_ERR_NOMEM (-4)  /* device or pinned-host allocation failed */
#define SHF_HB_ERR_ARCH (-5)   /* current device is not gfx950 (MI355X) */
#define SHF_HB_ERR_FORKED (-6) /* this process is a fork() child of one that had used the library (see "fork") */

/* Where the caller's buffers live. */
#define SHF_HASH_MEM_DEVICE 0 /* keys, offsets and out are device (HBM) pointers */
#define SHF_HASH_MEM_HOST 1   /* host pointers (pageable or pinned); pipelined through the process's staging slots (pageable fixed-length keys by the HIP runtime's own pageable copy), or read and written by the kernel in place (fixed-length keys in page-locked caller buffers); pageable memory is never page-locked by the library */

/* One result record: identical bytes to SHF_HASH (shf.private.h:180-185). */
typedef struct shf_hash128 {
    uint64_t h1; /* SHF_HASH.u64[0] */
    uint64_t h2; /* SHF_HASH.u64[1] */
} shf_hash128;

/* The hash bits put/find consume (shf.c:800-803, :893-896), packed in one u64:
 *   bits  0.. 7 win  = SHF_HASH.u16[0] % 256
 *   bits  8..18 tab  = SHF_HASH.u16[1] % 2048
 *   bits 19..27 row  = SHF_HASH.u16[2] % 512
 *   bits 28..31 0    (the SHF_UID `ref` field, chosen later by put)
 *   bits 32..52 rnd  = SHF_HASH.u32[2] % 2^21
 * i.e. the low word is SHF_UID.as_u32 (shf.private.h:170-178) with ref = 0. */
#define SHF_UID_PARTS_WIN(p) ((uint32_t)((p)&0xffu))
#define SHF_UID_PARTS_TAB(p) ((uint32_t)(((p) >> 8) & 0x7ffu))
#define SHF_UID_PARTS_ROW(p) ((uint32_t)(((p) >> 19) & 0x1ffu))
#define SHF_UID_PARTS_RND(p) ((uint32_t)(((p) >> 32) & 0x1fffffu))

/* ---- fixed-length keys: key i = keys[i*key_len .. (i+1)*key_len) ---------- */

/* Synchronous. mem = SHF_HASH_MEM_DEVICE or SHF_HASH_MEM_HOST; out = n records. */
SHF_HB_API int shf_hash_batch_fixed(const void *keys, uint32_t key_len, uint64_t n, uint32_t seed,
                         shf_hash128 *out, int mem);

/* Asynchronous, device-resident: enqueue on `hip_stream` (NULL = the null
 * stream) and return; results are valid once that stream has reached the
 * point of the call. */
SHF_HB_API int shf_hash_batch_fixed_async(const void *d_keys, uint32_t key_len, uint64_t n, uint32_t seed,
                               shf_hash128 *d_out, void *hip_stream);

/* ---- variable-length keys: key i = bytes[offsets[i] .. offsets[i+1]) ------- */
/* offsets has n + 1 monotone entries (64-bit, so batches may exceed 4 GiB). */

SHF_HB_API int shf_hash_batch_var(const void *bytes, const uint64_t *offsets, uint64_t n, uint32_t seed,
                       shf_hash128 *out, int mem);

SHF_HB_API int shf_hash_batch_var_async(const void *d_bytes, const uint64_t *d_offsets, uint64_t n, uint32_t seed,
                             shf_hash128 *d_out, void *hip_stream);

/* As shf_hash_batch_var_async, for a caller that knows the batch's packed byte
 * count key_bytes = offsets[n] - offsets[0] (whoever packed the keys does). The
 * mean key length sizes the LDS window of each 64-key span, so batches of
 * short keys keep more spans in flight per CU (U[8,128] B keys: 5.1 vs
 * 3.4 TB/s). A wrong key_bytes changes the speed, never the results. The
 * host-memory calls do this by themselves. (An extension: the reference hashes
 * one key at a time and has no such parameter.) */
SHF_HB_API int shf_hash_batch_var_sized_async(const void *d_bytes, const uint64_t *d_offsets, uint64_t n,
                                   uint64_t key_bytes, uint32_t seed, shf_hash128 *d_out, void *hip_stream);

/* ---- UID parts instead of the 16-byte hash (8 B per key, see above) -------
 *
 * The bits put/get/del read (shf.c:800-803, :893-896) and nothing else: 8 B per
 * key back instead of 16, e.g. over PCIe for host buffers. A host caller feeds
 * them to the reference's caller-supplied-hash seam with shf_use_uid_parts()
 * (shf_hash_batch_shf.h), which rebuilds every byte of SHF_HASH that shf.c reads.
 * Synchronous forms: mem = SHF_HASH_MEM_DEVICE or SHF_HASH_MEM_HOST, as
 * shf_hash_batch_fixed / _var (same staging pool, copy threads, variable-length
 * checks and status codes); parts = n words. */
SHF_HB_API int shf_uid_parts_batch_fixed(const void *keys, uint32_t key_len, uint64_t n, uint32_t seed,
                                         uint64_t *parts, int mem);
SHF_HB_API int shf_uid_parts_batch_var(const void *bytes, const uint64_t *offsets, uint64_t n, uint32_t seed,
                                       uint64_t *parts, int mem);

SHF_HB_API int shf_uid_parts_batch_fixed_async(const void *d_keys, uint32_t key_len, uint64_t n, uint32_t seed,
                                    uint64_t *d_parts, void *hip_stream);
SHF_HB_API int shf_uid_parts_batch_var_async(const void *d_bytes, const uint64_t *d_offsets, uint64_t n, uint32_t seed,
                                  uint64_t *d_parts, void *hip_stream);

/* ---- several GPUs: host buffers in and out, keys split into n_devices even
 * index ranges, one host thread and one device per range, no collective.
 * n_devices <= 0 means every visible device. ------------------------------ */

SHF_HB_API int shf_hash_batch_fixed_multi(const void *keys, uint32_t key_len, uint64_t n, uint32_t seed,
                               shf_hash128 *out, int n_devices);
SHF_HB_API int shf_hash_batch_var_multi(const void *bytes, const uint64_t *offsets, uint64_t n, uint32_t seed,
                             shf_hash128 *out, int n_devices);
/* The same with 8-B UID parts out instead of 16-B records (see "UID parts"). */
SHF_HB_API int shf_uid_parts_batch_fixed_multi(const void *keys, uint32_t key_len, uint64_t n, uint32_t seed,
                                               uint64_t *parts, int n_devices);
SHF_HB_API int shf_uid_parts_batch_var_multi(const void *bytes, const uint64_t *offsets, uint64_t n, uint32_t seed,
                                             uint64_t *parts, int n_devices);

/* ---- kernel selection (tests and benchmarks) ------------------------------- */
#define SHF_HB_KERNEL_AUTO 0    /* what every function above uses */
#define SHF_HB_KERNEL_FIXED16 1 /* key_len == 16, 16-B aligned keys */
#define SHF_HB_KERNEL_TILED 2   /* key_len % 16 == 0, >= 32, 16-B aligned keys */
#define SHF_HB_KERNEL_GENERIC 3 /* any key_len, any alignment, per-lane loads straight from HBM */
#define SHF_HB_KERNEL_SPAN 4    /* key_len <= 318 (fixed) / any keys (var): LDS-staged spans */
#define SHF_HB_KERNEL_ROUND 5   /* var only: keys streamed 128 B per round through LDS */
#define SHF_HB_KERNEL_SPAN_PP 6 /* var only: LDS-staged spans, two tiles per window in turn (what AUTO uses for
                                   spans over 10 KiB or an unknown byte count); not for probes */

SHF_HB_API int shf_hash_batch_fixed_kernel_async(const void *d_keys, uint32_t key_len, uint64_t n, uint32_t seed,
                                      shf_hash128 *d_out, int kernel, void *hip_stream);
/* kernel: SHF_HB_KERNEL_AUTO, SHF_HB_KERNEL_SPAN, SHF_HB_KERNEL_SPAN_PP, SHF_HB_KERNEL_ROUND or
 * SHF_HB_KERNEL_GENERIC */
SHF_HB_API int shf_hash_batch_var_kernel_async(const void *d_bytes, const uint64_t *d_offsets, uint64_t n,
                                    uint32_t seed, shf_hash128 *d_out, int kernel, void *hip_stream);
SHF_HB_API int shf_hash_batch_var_sized_kernel_async(const void *d_bytes, const uint64_t *d_offsets, uint64_t n,
                                          uint64_t key_bytes, uint32_t seed, shf_hash128 *d_out, int kernel,
                                          void *hip_stream);

/* ---- row pre-probe ----------------------------------------
 *
 * The first half of shf_find_key_internal() (/root/reference/src/shf.c:886-922)
 * for a whole batch: hash each key, pick its window, tab and row, and scan the
 * row's 16 refs for the ones whose pos != 0, rnd and tab match (shf.c:919-921),
 * against a copy of the store's rows kept in HBM (a "row index"). What is left
 * for the CPU is the key compare and the value copy at the returned pos.
 *
 * The index is a snapshot: rows change under put/del/part/shrink, so a result
 * is a hint to verify (the key compare does that) and a key with no candidate
 * goes through the ordinary shf_get_key_val_*() path. INTEGRATION.md §6 shows
 * the exporter a maintainer adds to shf.c and the resulting get loop.
 *
 * Index layout (device memory owned by the shf_row_index handle):
 *   tab_slot[(win << 11) | tab2] = (slot << 11) | tab, or SHF_PROBE_NONE
 *       tab  = SHF_WIN_MMAP.tabs[tab2].tab of window win (shf.private.h:85,
 *              read at shf.c:806 / :906), i.e. which physical tab holds tab2's refs;
 *       slot = which 64-KiB block of `rows` holds that tab's rows.
 *       SHF_ROW_INDEX_TABS = 256 * 2048 entries.
 *   rows[slot] = SHF_TAB_MMAP.row[0..511] of that tab (shf.private.h:59-66),
 *       byte for byte: 512 rows x 16 refs x 8 B, ref = SHF_REF_MMAP
 *       {u32 tab:11 | rnd:21 << 11, u32 pos} (shf.private.h:48-52). */
#define SHF_PROBE_NONE 0xffffffffu        /* = SHF_UID_NONE (shf.h:354) */
#define SHF_ROW_INDEX_TABS (256u * 2048u) /* tab_slot entries */
#define SHF_ROW_INDEX_SLOT_BYTES 65536u   /* 512 rows x 128 B */

/* One probe result per key. */
typedef struct shf_probe {
    uint32_t uid;  /* SHF_UID.as_u32 (win | tab2 << 8 | row << 19 | ref << 28, shf.private.h:170-178)
                      of the first candidate ref, or SHF_PROBE_NONE; this is the shf_uid a successful
                      get returns when the first candidate's key matches */
    uint32_t pos;  /* that ref's pos: offset of its key,value record in the tab (0 if none) */
    uint16_t mask; /* bit r set: ref r of the row is a candidate (pos != 0, rnd, tab2 match) */
    uint16_t tab;  /* physical tab (wins[win].tabs[tab2].tab), 0xffff if the window/tab is not indexed */
    uint32_t slot; /* rows slot scanned, SHF_PROBE_NONE if none */
} shf_probe;

typedef struct shf_row_index shf_row_index; /* opaque; lives on the device current at create */

/* Allocate an index of n_slots row blocks on the current device: every
 * tab_slot entry SHF_PROBE_NONE, every row empty. */
SHF_HB_API int shf_row_index_create(uint64_t n_slots, shf_row_index **out);
SHF_HB_API int shf_row_index_destroy(shf_row_index *index);
/* Copy SHF_ROW_INDEX_TABS entries (host or device memory) into the index
 * (entries naming a slot >= n_slots are treated as absent by the probes).
 * Synchronous; it also makes the probes' compact copy of the map (a 1-B rank
 * per entry among its window's distinct entries, plus those entries: 768 KiB
 * that stay in L2 where the 2-MiB map does not). */
SHF_HB_API int shf_row_index_set_tabs(shf_row_index *index, const uint32_t *tab_slot);
/* Copy count row blocks (count * 64 KiB, host or device memory) into slots
 * [first, first + count). Synchronous. */
SHF_HB_API int shf_row_index_set_rows(shf_row_index *index, uint64_t first, uint64_t count, const void *rows);
/* Device pointers of the index, for producers that fill it on the device.
 * From this call on the probes read tab_slot itself (the compact copy made by
 * set_tabs could go stale), so device-side writes are seen by the next probe. */
SHF_HB_API int shf_row_index_device_ptrs(const shf_row_index *index, uint32_t **d_tab_slot, void **d_rows,
                                         uint64_t *n_slots);

/* Hash and probe device-resident keys (same key layouts as above). d_hashes
 * may be NULL; if not, it receives the n SHF_HASH records as well. */
SHF_HB_API int shf_probe_batch_fixed_async(const shf_row_index *index, const void *d_keys, uint32_t key_len,
                                           uint64_t n, uint32_t seed, shf_hash128 *d_hashes, shf_probe *d_probe,
                                           void *hip_stream);
SHF_HB_API int shf_probe_batch_var_async(const shf_row_index *index, const void *d_bytes,
                                         const uint64_t *d_offsets, uint64_t n, uint32_t seed,
                                         shf_hash128 *d_hashes, shf_probe *d_probe, void *hip_stream);
/* Synchronous, like shf_hash_batch_fixed / _var: mem = SHF_HASH_MEM_DEVICE
 * (every buffer in HBM) or SHF_HASH_MEM_HOST (keys, offsets, hashes and probes
 * in host memory, pipelined through pinned staging like the hashing calls).
 * hashes may be NULL. The index lives on the calling thread's current device. */
SHF_HB_API int shf_probe_batch_fixed(const shf_row_index *index, const void *keys, uint32_t key_len, uint64_t n,
                                     uint32_t seed, shf_hash128 *hashes, shf_probe *probes, int mem);
SHF_HB_API int shf_probe_batch_var(const shf_row_index *index, const void *bytes, const uint64_t *offsets,
                                   uint64_t n, uint32_t seed, shf_hash128 *hashes, shf_probe *probes, int mem);
/* Probe precomputed hashes (n records on the device). */
SHF_HB_API int shf_probe_batch_hashes_async(const shf_row_index *index, const shf_hash128 *d_hashes, uint64_t n,
                                            shf_probe *d_probe, void *hip_stream);
/* Fixed-length probe with a forced hashing kernel (tests and benchmarks). */
SHF_HB_API int shf_probe_batch_fixed_kernel_async(const shf_row_index *index, const void *d_keys,
                                                  uint32_t key_len, uint64_t n, uint32_t seed,
                                                  shf_hash128 *d_hashes, shf_probe *d_probe, int kernel,
                                                  void *hip_stream);

/* ---- tab part / shrink copy ------------------------------
 *
 * The two places the reference re-packs a tab's key,value data:
 *   shf_tab_part()   /root/reference/src/shf.c:722-779: a full tab's window map
 *                    sends every second tab2 naming it to a new tab (:683-692,
 *                    shf_tab_part_redirect below), every ref whose tab2 now
 *                    names the new tab is copied into it, then
 *   shf_tab_shrink() /root/reference/src/shf.c:678-720: the old tab is
 *                    re-created holding only its remaining refs' data.
 * A job takes one tab image (the bytes of a tab file: SHF_TAB_MMAP header,
 * 512 rows x 16 refs, data; shf.private.h:48-68) and writes the image of the
 * shrunk tab ("keep": refs that stay) and, for a part, of the new tab
 * ("move": refs whose tab2 the job's map sends to tab_new), byte for byte what
 * the reference's part / shrink leave in those files: header, all rows (a ref
 * not copied is 0), records appended in row/ref order. Bytes of an output past
 * its tab_used are not written.
 *
 * Reference quirks kept as they are: tab_refs_used counts each copied ref
 * twice (SHF_TAB_APPEND, shf.c:608, and SHF_TAB_REF_COPY, :651); the
 * SHF_DATA_TYPE byte at each copied record has an uninitialised `extended`
 * bit (shf.c:593-596), so the reference writes 0x3e or 0xbe depending on its
 * stack: the job names the byte to write per output. */
#define SHF_TAB_NONE 0xffffu /* tab_new of a shrink-only job */

typedef struct shf_tab_job {
    uint64_t src;       /* byte offset of the source tab image in the source buffer (8-B aligned) */
    uint64_t src_len;   /* its bytes (the tab file's size; at least its tab_used) */
    uint64_t keep;      /* byte offset of the keep (shrunk tab) output image in the output buffer (8-B aligned) */
    uint64_t move;      /* byte offset of the move (new tab) output image (8-B aligned); unused if tab_new is NONE */
    uint64_t cap;       /* bytes available at keep and at move each (>= 65560) */
    uint32_t map;       /* index of this job's 2048-entry tab2 -> tab map (after the redirect) */
    uint16_t tab_new;   /* the new tab's number, or SHF_TAB_NONE: shrink only */
    uint8_t keep_type;  /* SHF_DATA_TYPE byte written at each record copied to keep (0x3e: key and value STR32) */
    uint8_t move_type;  /* ... copied to move */
    int32_t status;     /* out: SHF_HB_OK, or SHF_HB_ERR_ARG (out of range, corrupt record, output too small);
                           after ERR_ARG the job's output images are unspecified (never written past cap) */
    uint32_t reserved;
} shf_tab_job;

typedef struct shf_tab_params {
    uint32_t fixed;              /* nonzero: a fixed-length store (SHF.is_fixed_key_val_len) */
    uint32_t fixed_key_len;      /* its key and value lengths (shf_set_is_fixed_len) */
    uint32_t fixed_val_len;
    uint32_t data_needed_factor; /* the tab growth factor (shf_set_data_need_factor; 0 = the default 1) */
} shf_tab_params;

/* Device-resident: every buffer in HBM (jobs too: their status is written
 * back there). src_bytes / dst_bytes / n_maps bound what the jobs may name. */
SHF_HB_API int shf_tab_copy_batch_async(const void *d_src, uint64_t src_bytes, void *d_dst, uint64_t dst_bytes,
                                        shf_tab_job *d_jobs, uint32_t n_jobs, const uint16_t *d_maps,
                                        uint32_t n_maps, const shf_tab_params *params, void *hip_stream);
/* Synchronous: mem = SHF_HASH_MEM_DEVICE (every buffer in HBM) or
 * SHF_HASH_MEM_HOST (host buffers, copied through the device; dst keeps the
 * bytes the copy does not write). Returns SHF_HB_ERR_ARG if any job failed
 * (see its status). */
SHF_HB_API int shf_tab_copy_batch(const void *src, uint64_t src_bytes, void *dst, uint64_t dst_bytes,
                                  shf_tab_job *jobs, uint32_t n_jobs, const uint16_t *maps, uint32_t n_maps,
                                  const shf_tab_params *params, int mem);
/* shf_tab_part()'s redirect of a window's 2048-entry tab2 -> tab map (host
 * memory, shf.c:683-692): of the entries naming tab_old, every second one
 * (the 2nd, 4th, ...) now names tab_new. */
SHF_HB_API int shf_tab_part_redirect(uint16_t *map, uint32_t tab_old, uint32_t tab_new);

/* ---- window order of a batch ("sorting a batch by win") ---
 *
 * perm[0..n) = the key indices 0..n-1 stably sorted by the window each key's
 * hash selects, win = h1 & 0xff (the put/get bit consumer,
 * /root/reference/src/shf.c:800, :893): window 0's keys first, each window's
 * keys in batch order. win_start (optional, 257 entries) = the position in
 * perm of each window's first key, then n.
 * Everything a put/get/del touches belongs to its key's window (the window's
 * lock, tab2 -> tab map, tabs and tab files; new tabs are numbered per window,
 * shf.c:432), so running a batch's puts/gets/dels in perm order leaves the
 * store byte for byte as batch order does, uids included, while consecutive
 * operations find their window's structures in cache (INTEGRATION.md §8;
 * shf_put_batch_var_win_ordered in shf_hash_batch_shf.h).
 * n < 2^32 (32-bit indices); n == 0 sets win_start to zeros.
 *
 * _async: every pointer on the device, enqueued on hip_stream; d_workspace of
 * at least shf_win_order_workspace_bytes(n) bytes, 16-B aligned (else
 * SHF_HB_ERR_ARG), in use until the call has run on the stream. Not reentrant
 * on one workspace.
 * shf_win_order: synchronous; mem = SHF_HASH_MEM_DEVICE (device pointers; runs
 * on the null stream, after the caller's work there, like the synchronous
 * hashing calls) or SHF_HASH_MEM_HOST (host pointers, copied through device
 * buffers). Its workspace is kept per thread and device across calls. */
SHF_HB_API size_t shf_win_order_workspace_bytes(uint64_t n);
SHF_HB_API int shf_win_order_async(const shf_hash128 *d_hashes, uint64_t n, uint32_t *d_perm,
                                   uint32_t *d_win_start, void *d_workspace, size_t workspace_bytes,
                                   void *hip_stream);
SHF_HB_API int shf_win_order(const shf_hash128 *hashes, uint64_t n, uint32_t *perm, uint32_t *win_start, int mem);

/* ---- hash + window order in one call ("alongside") -------
 *
 * The 16-B records of shf_hash_batch_fixed_async / shf_hash_batch_var_async in
 * d_out, and their window order in d_perm / d_win_start exactly as
 * shf_win_order_async would compute it from d_out -- without reading d_out
 * back: the hashing kernel writes each key's window byte beside its record
 * into the workspace (for 16-B keys it instead ranks each 4096-key chunk by
 * window itself and writes the chunk's counts and order), and the order passes
 * work from those. d_workspace: at least
 * shf_win_order_workspace_bytes(n) bytes, 16-B aligned. n < 2^32. Enqueued on
 * hip_stream like the other _async calls; variable-length key errors are
 * reported by shf_hash_batch_status() (an invalid key's record is not written
 * and its window byte is then unspecified, so perm is too). */
SHF_HB_API int shf_hash_batch_fixed_win_async(const void *d_keys, uint32_t key_len, uint64_t n, uint32_t seed,
                                              shf_hash128 *d_out, uint32_t *d_perm, uint32_t *d_win_start,
                                              void *d_workspace, size_t workspace_bytes, void *hip_stream);
SHF_HB_API int shf_hash_batch_var_win_async(const void *d_bytes, const uint64_t *d_offsets, uint64_t n,
                                            uint32_t seed, shf_hash128 *d_out, uint32_t *d_perm,
                                            uint32_t *d_win_start, void *d_workspace, size_t workspace_bytes,
                                            void *hip_stream);
/* Synchronous forms: mem = SHF_HASH_MEM_DEVICE (every pointer on the device)
 * or SHF_HASH_MEM_HOST (keys, offsets, out, perm and win_start in host memory:
 * the records come back through the hashing pipeline while each key's window
 * byte stays on the device, so they are never copied back in to be ordered --
 * hash + shf_win_order(SHF_HASH_MEM_HOST) move 16 + 4 B per key more over PCIe).
 * win_start may be NULL. The workspace is the library's, kept per thread and
 * device. Variable-length keys with invalid offsets: SHF_HB_ERR_ARG (host memory:
 * checked before anything is copied). */
SHF_HB_API int shf_hash_batch_fixed_win(const void *keys, uint32_t key_len, uint64_t n, uint32_t seed,
                                        shf_hash128 *out, uint32_t *perm, uint32_t *win_start, int mem);
SHF_HB_API int shf_hash_batch_var_win(const void *bytes, const uint64_t *offsets, uint64_t n, uint32_t seed,
                                      shf_hash128 *out, uint32_t *perm, uint32_t *win_start, int mem);
/* UID parts + window order in one call: parts[] as shf_uid_parts_batch_fixed /
 * _var, perm / win_start exactly as shf_win_order computes them from the
 * batch's hashes (the window is SHF_UID_PARTS_WIN(parts[i]) = h1 & 0xff). With
 * host memory 8 B of parts + 4 B of order per key cross PCIe back, instead of
 * 16 + 4 (a window-ordered put from parts). mem, win_start
 * and errors as shf_hash_batch_fixed_win / _var_win. */
SHF_HB_API int shf_uid_parts_batch_fixed_win(const void *keys, uint32_t key_len, uint64_t n, uint32_t seed,
                                             uint64_t *parts, uint32_t *perm, uint32_t *win_start, int mem);
SHF_HB_API int shf_uid_parts_batch_var_win(const void *bytes, const uint64_t *offsets, uint64_t n, uint32_t seed,
                                           uint64_t *parts, uint32_t *perm, uint32_t *win_start, int mem);
/* The same with a forced hashing kernel (tests and benchmarks; SHF_HB_KERNEL_*). */
SHF_HB_API int shf_hash_batch_fixed_win_kernel_async(const void *d_keys, uint32_t key_len, uint64_t n,
                                                     uint32_t seed, shf_hash128 *d_out, uint32_t *d_perm,
                                                     uint32_t *d_win_start, void *d_workspace,
                                                     size_t workspace_bytes, int kernel, void *hip_stream);
SHF_HB_API int shf_hash_batch_var_win_kernel_async(const void *d_bytes, const uint64_t *d_offsets, uint64_t n,
                                                   uint32_t seed, shf_hash128 *d_out, uint32_t *d_perm,
                                                   uint32_t *d_win_start, void *d_workspace,
                                                   size_t workspace_bytes, int kernel, void *hip_stream);

/* ---- status of asynchronous variable-length calls -------------------------
 * Waits for hip_stream (NULL = the null stream), then returns SHF_HB_ERR_ARG if
 * any asynchronous variable-length call (hashing, UID parts or probe) that
 * this thread enqueued on its current device since the previous query met an
 * invalid key (see Conventions), else SHF_HB_OK; the query clears the flag
 * (read and cleared in one device-side exchange, so a call still running on
 * another stream that flags a key after the read is reported by a later query,
 * never lost). */
SHF_HB_API int shf_hash_batch_status(void *hip_stream);

/* ---- info ----------------------------------------------------------------- */
SHF_HB_API int shf_hash_batch_device_count(void);          /* visible HIP devices, or a negative status */
SHF_HB_API int shf_hash_batch_check_device(void);          /* SHF_HB_OK if the current device can run the kernels */
SHF_HB_API int shf_hash_batch_last_hip_error(void);        /* last hipError_t seen by this thread */
/* Frees the calling thread's per-device state (stream, status words, window-order
 * buffers), the state exited threads left for reuse, and every idle staging slot
 * of the process's pools; what other live threads hold is kept. Any later call
 * starts afresh. */
SHF_HB_API int shf_hash_batch_release(void);
SHF_HB_API const char *shf_hash_batch_strerror(int status);
SHF_HB_API const char *shf_hash_batch_version(void);

#ifdef __cplusplus
}
#endif
#endif /* SHF_HASH_BATCH_H */
