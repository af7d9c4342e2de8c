/*
 * shf_hash_batch_ceiling.h -- measurement kernels of the bench-only library
 * libshf_hb_bench.so (NOT the product libshf_hash_batch.so, which neither
 * contains nor exports them; only bench.py, tools/ and the tests load this
 * one): the on-box HBM ceilings that bench.py reports each
 * hashing kernel against (roofline.frac_of_copy_ceiling), and the access
 * patterns that calibrate rocprofv3's FETCH_SIZE for the probe's row gathers
 * and the tab copy's unaligned loads. They replace no reference interface:
 * the reference has no device code. Each kernel moves exactly the bytes of one
 * hashing kernel's pattern and computes only an XOR fold of what it reads.
 */
#ifndef SHF_HASH_BATCH_CEILING_H
#define SHF_HASH_BATCH_CEILING_H

#include <stdint.h>

#include "shf_hash_batch.h"

#ifdef __cplusplus
extern "C" {
#endif

/* kind: bytes moved per lane (n lanes per launch) */
#define SHF_HB_CEIL_COPY 0      /* 16-B nt load src[i] + 16-B store dst[i]: k_fixed16's shape, 32 B (src 16-B aligned) */
#define SHF_HB_CEIL_READ16 1    /* 16 x 16-B nt loads (a wave reads one contiguous 16 KiB) + 16-B store: 272 B;
                                   n a multiple of 64, src_bytes >= 256 n */
#define SHF_HB_CEIL_GATHER128 2 /* 4-B idx[i], the 128-B row src[128 idx[i] ..], fetched 8 lanes per row like the
                                   row pre-probe, + 16-B store: 148 B; an idx[i] >= src_bytes / 128 reads row 0 */
#define SHF_HB_CEIL_STREAM16U 3 /* 16-B load at src + 16 i + shift (byte-unaligned: shift = 7 for an aligned src)
                                   + 16-B store: 32 B; src_bytes >= 16 n + 16 */
#define SHF_HB_CEIL_VALU_ADD 4  /* no loads: 8 independent v_add_u32 chains per lane, src_bytes rounds (the loop
                                   count; d_src any non-NULL value, not read), one 16-B store: a VALU-saturating
                                   launch of full-rate instructions (8 x src_bytes per lane) */
#define SHF_HB_CEIL_VALU_MUL 5  /* the same with v_mul_lo_u32 (half rate on gfx950) */
#define SHF_HB_CEIL_COPY4 6     /* SHF_HB_CEIL_COPY's bytes, 4 x 16 B per lane (1024 units per 256-thread block) */
/* the same bytes as SHF_HB_CEIL_COPY, other instruction choices (the sweep that picks the ceiling) */
#define SHF_HB_CEIL_COPY_PLAIN 7 /* plain loads */
#define SHF_HB_CEIL_COPY_NT 8    /* nontemporal loads and stores */
#define SHF_HB_CEIL_COPY_SLEEP 9 /* nontemporal loads, a short s_sleep before the store */
#define SHF_HB_CEIL_COPY2 10     /* two 16-B units per lane */
#define SHF_HB_CEIL_READ16_NT 11 /* SHF_HB_CEIL_READ16 with a nontemporal store */
#define SHF_HB_CEIL_READ16_W1 12 /* SHF_HB_CEIL_READ16_NT launched one wave (64 lanes) per workgroup */
#define SHF_HB_CEIL_PROBE_ROWS 13 /* SHF_HB_CEIL_GATHER128 with the index as 16-B records (row in the first word,
                                     d_idx 16-B aligned), a nontemporal store and the probe kernel's 32 KiB of LDS
                                     per workgroup (its occupancy): the probe's 160 B per lane */

/* Enqueue one launch on hip_stream. Device pointers; dst 16-B aligned, n x 16 B. */
SHF_HB_API int shf_hb_ceiling_async(int kind, const void *d_src, uint64_t src_bytes, const uint32_t *d_idx,
                                    void *d_dst, uint64_t n, void *hip_stream);

/* *dev = the device address of page-locked host memory (hipHostGetDevicePointer), so that a ceiling kernel
 * can read or write host memory over PCIe as the product's zero copy does; SHF_HB_ERR_ARG if not mappable. */
SHF_HB_API int shf_hb_host_device_ptr(const void *host, void **dev);

#ifdef __cplusplus
}
#endif
#endif /* SHF_HASH_BATCH_CEILING_H */
