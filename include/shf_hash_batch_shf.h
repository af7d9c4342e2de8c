/*
 * shf_hash_batch_shf.h -- the GPU batch hashes (shf_hash_batch.h) fed into
 * SharedHashFile's unchanged put/get/del flow.
 *
 * The reference hashes one key per call, shf_make_hash(key, key_len)
 * (/root/reference/src/shf.c:450-462), leaving the result in thread-locals that
 * put/get/del read (SHF_HASH shf_hash, shf_hash_key, shf_hash_key_len:
 * /root/reference/src/shf.private.h:187-189). Its tests already set those by
 * hand for caller-supplied hashes (/root/reference/src/test.9.shf.c:176-182);
 * this header packages that seam:
 *
 *   shf_use_hash()           the three assignments, from one shf_hash128 record
 *   shf_use_uid_parts()      the same from an 8-B UID-parts word
 *                            (shf_uid_parts_batch_*): the SHF_HASH bytes shf.c
 *                            reads, rebuilt; put/get/del behave identically
 *   shf_put_batch_var()      INTEGRATION.md §3: hash a host batch on the GPU,
 *                            then shf_put_key_val() per key
 *   shf_put_batch_var_parts()  the same with UID parts: 8 B per key back
 *                            from the GPU instead of 16
 *   shf_get_batch_probed()   INTEGRATION.md §6: a get batch driven by row
 *                            pre-probe records, falling back to the ordinary
 *                            get with the batch hash
 *   shf_put_batch_var_parts_win_ordered()
 *                            the window-ordered put from UID parts
 *   shf_put_batch_var_win_ordered(), shf_get_batch_win_ordered()
 *                            the same put / get loops run in
 *                            the GPU's window order (shf_win_order): the store
 *                            ends byte for byte as in batch order, each
 *                            window's structures are met while in cache
 *   shf_put_batch_win_range()  one worker process's share of a window-ordered
 *                            batch: whole windows, no lock shared with others
 *
 * Include it after the reference's shf.private.h and shf.h, in that order
 * (shf.h names the types shf.private.h defines). Everything is static inline:
 * SharedHashFile.a gains no symbol, the application links libshf_hash_batch.so
 * and nothing else.
 */
#ifndef SHF_HASH_BATCH_SHF_H
#define SHF_HASH_BATCH_SHF_H

#ifndef __SHF_PRIVATE_H__
#error "include the reference's shf.private.h and shf.h before shf_hash_batch_shf.h"
#endif

#include <stdlib.h>
#include <string.h>

#include "shf_hash_batch.h"

/* shf_make_hash(key, key_len) with the hash already computed (h = that key's
 * record from a shf_hash_batch_* call). The key pointer is kept, not copied,
 * exactly as shf_make_hash() keeps it (shf.c:460-461): it must stay valid
 * until the put/get/del that follows. */
static inline void shf_use_hash(const char *key, uint32_t key_len, const shf_hash128 *h)
{
    shf_hash.u64[0] = h->h1;
    shf_hash.u64[1] = h->h2;
    shf_hash_key = key;
    shf_hash_key_len = key_len;
}

/* shf_make_hash(key, key_len) from a UID-parts word (shf_uid_parts_batch_*,
 * shf_hash_batch.h): put and find read only SHF_HASH.u16[0] % 256 (win),
 * u16[1] % 2048 (tab2), u16[2] % 512 (row) and u32[2] % 2^21 (rnd)
 * (/root/reference/src/shf.c:800-803, :893-896), so those four fields get the
 * parts' values and every other byte is 0: each put/get/del then takes the same
 * window, tab, row and rnd -- the same store bytes and shf_uid -- as with the
 * full hash. (Anything else reading shf_hash -- only a debug build's trace,
 * shf.c:461 -- sees the zeros.) The key pointer is kept, as by shf_use_hash. */
static inline void shf_use_uid_parts(const char *key, uint32_t key_len, uint64_t parts)
{
    shf_hash.u64[0] = 0;
    shf_hash.u64[1] = 0;
    shf_hash.u16[0] = (uint16_t)SHF_UID_PARTS_WIN(parts);
    shf_hash.u16[1] = (uint16_t)SHF_UID_PARTS_TAB(parts);
    shf_hash.u16[2] = (uint16_t)SHF_UID_PARTS_ROW(parts);
    shf_hash.u32[2] = SHF_UID_PARTS_RND(parts);
    shf_hash_key = key;
    shf_hash_key_len = key_len;
}

/* Put n host keys (key i = bytes[offsets[i] .. offsets[i+1])) with values
 * (value i = vals[val_offsets[i] .. val_offsets[i+1])): one GPU batch hash
 * (shf_hash_batch_var, SHF_HASH_MEM_HOST, seed 12345), then the reference's
 * shf_put_key_val() per key. Returns the number of keys put (n, or the index
 * of the first put that did not return SHF_RET_KEY_PUT), or a negative
 * SHF_HB_ERR_* status with nothing put. */
static inline int64_t shf_put_batch_var(SHF *shf, const char *bytes, const uint64_t *offsets, uint64_t n,
                                        const char *vals, const uint64_t *val_offsets)
{
    if (n == 0) return 0;
    shf_hash128 *h = (shf_hash128 *)malloc(n * sizeof *h);
    if (!h) return SHF_HB_ERR_NOMEM;
    const int rc = shf_hash_batch_var(bytes, offsets, n, SHF_HASH_BATCH_SEED, h, SHF_HASH_MEM_HOST);
    if (rc != SHF_HB_OK) {
        free(h);
        return rc;
    }
    uint64_t i = 0;
    for (; i < n; ++i) {
        shf_use_hash(bytes + offsets[i], (uint32_t)(offsets[i + 1] - offsets[i]), &h[i]);
        if (shf_put_key_val(shf, vals + val_offsets[i], (uint32_t)(val_offsets[i + 1] - val_offsets[i])) !=
            SHF_RET_KEY_PUT)
            break;
    }
    free(h);
    return (int64_t)i;
}

/* shf_put_batch_var() with UID parts: one GPU batch (shf_uid_parts_batch_var,
 * SHF_HASH_MEM_HOST: 8 B per key back over PCIe), then shf_use_uid_parts() +
 * shf_put_key_val() per key; the store ends byte for byte as after
 * shf_put_batch_var(). uids_out (optional, n entries): shf_uid after each put.
 * Returns as shf_put_batch_var(). */
static inline int64_t shf_put_batch_var_parts(SHF *shf, const char *bytes, const uint64_t *offsets, uint64_t n,
                                              const char *vals, const uint64_t *val_offsets, uint32_t *uids_out)
{
    if (n == 0) return 0;
    uint64_t *parts = (uint64_t *)malloc(n * sizeof *parts);
    if (!parts) return SHF_HB_ERR_NOMEM;
    const int rc = shf_uid_parts_batch_var(bytes, offsets, n, SHF_HASH_BATCH_SEED, parts, SHF_HASH_MEM_HOST);
    if (rc != SHF_HB_OK) {
        free(parts);
        return rc;
    }
    uint64_t i = 0;
    for (; i < n; ++i) {
        shf_use_uid_parts(bytes + offsets[i], (uint32_t)(offsets[i + 1] - offsets[i]), parts[i]);
        if (shf_put_key_val(shf, vals + val_offsets[i], (uint32_t)(val_offsets[i + 1] - val_offsets[i])) !=
            SHF_RET_KEY_PUT)
            break;
        if (uids_out) uids_out[i] = shf_uid;
    }
    free(parts);
    return (int64_t)i;
}

/* Get n host keys, given their hashes and row pre-probe records (from
 * shf_probe_batch_var / _fixed against a row index of this store):
 *   a candidate ref  -> shf_get_uid_val_copy(uid) (shf.c:1037, which checks
 *                       the ref's pos and tab but not the key), then the
 *                       stored key is compared with key i;
 *   otherwise        -> shf_get_key_val_copy() with the batch hash in the
 *                       seam: found or not, exactly as the reference decides.
 * The index is a snapshot, so a stale candidate only costs the fast path.
 * For every key found, shf_val / shf_val_len hold its value when on_found(ctx, i)
 * is called. Returns the keys found; *fast (if not NULL) = those served by the
 * uid path.
 *
 * Concurrency: shf_get_uid_val_copy() copies the value under the window's
 * reader lock and releases it; the uid path then reads the stored key's length
 * word (shf_key_addr - 4) and bytes WITHOUT that lock, whereas the reference's
 * own get compares keys under it (shf.c:933-934). If another thread or process
 * may delete, re-put or part the same window while this runs, a ref whose
 * record was replaced in between could pair the old value with a matching new
 * key. Use the uid path on stores that are quiescent for writers during the
 * batch (bulk-read phases); otherwise pass probes whose mask is 0 (every key
 * then takes the locked shf_get_key_val_copy() with the batch hash). */
static inline uint64_t shf_get_batch_probed(SHF *shf, const char *bytes, const uint64_t *offsets, uint64_t n,
                                            const shf_hash128 *hashes, const shf_probe *probes,
                                            void (*on_found)(void *ctx, uint64_t i), void *ctx, uint64_t *fast)
{
    uint64_t found = 0, f = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const char *k = bytes + offsets[i];
        const uint32_t kl = (uint32_t)(offsets[i + 1] - offsets[i]);
        if (probes[i].mask && shf_get_uid_val_copy(shf, probes[i].uid) == SHF_RET_KEY_FOUND) {
            uint32_t stored_len = shf->fixed_key_len; /* fixed-length stores keep no length (shf.c:927) */
            if (!shf->is_fixed_key_val_len) memcpy(&stored_len, (const char *)shf_key_addr - 4, 4);
            if (stored_len == kl && memcmp(shf_key_addr, k, kl) == 0) {
                ++found;
                ++f;
                if (on_found) on_found(ctx, i);
                continue;
            }
        }
        shf_use_hash(k, kl, &hashes[i]);
        if (shf_get_key_val_copy(shf) == SHF_RET_KEY_FOUND) {
            ++found;
            if (on_found) on_found(ctx, i);
        }
    }
    if (fast) *fast = f;
    return found;
}

/* shf_put_batch_var() in window order: one GPU call hashes the batch and
 * orders it by window (shf_hash_batch_var_win: only the records and the order
 * cross PCIe), then shf_put_key_val() per key in that order. Keys of one window keep their batch order and windows share no
 * state, so the store (files, uids) ends exactly as shf_put_batch_var() leaves
 * it. Returns n, the number of puts made before the first one that did not
 * return SHF_RET_KEY_PUT (in window order: which keys went in is then
 * perm[0 .. returned)), or a negative SHF_HB_ERR_* status with nothing put.
 * perm_out (optional, n entries): the order used. */
static inline int64_t shf_put_batch_var_win_ordered(SHF *shf, const char *bytes, const uint64_t *offsets, uint64_t n,
                                                    const char *vals, const uint64_t *val_offsets,
                                                    uint32_t *perm_out)
{
    if (n == 0) return 0;
    shf_hash128 *h = (shf_hash128 *)malloc(n * sizeof *h);
    uint32_t *perm = perm_out ? perm_out : (uint32_t *)malloc(n * sizeof *perm);
    if (!h || !perm) {
        free(h);
        if (!perm_out) free(perm);
        return SHF_HB_ERR_NOMEM;
    }
    int rc = shf_hash_batch_var_win(bytes, offsets, n, SHF_HASH_BATCH_SEED, h, perm, NULL, SHF_HASH_MEM_HOST);
    uint64_t j = 0;
    if (rc == SHF_HB_OK)
        for (; j < n; ++j) {
            const uint64_t i = perm[j];
            shf_use_hash(bytes + offsets[i], (uint32_t)(offsets[i + 1] - offsets[i]), &h[i]);
            if (shf_put_key_val(shf, vals + val_offsets[i], (uint32_t)(val_offsets[i + 1] - val_offsets[i])) !=
                SHF_RET_KEY_PUT)
                break;
        }
    free(h);
    if (!perm_out) free(perm);
    return rc == SHF_HB_OK ? (int64_t)j : rc;
}

/* shf_put_batch_var_win_ordered() with UID parts: one GPU call
 * (shf_uid_parts_batch_var_win, host memory: 8 B of parts + 4 B of order per
 * key cross PCIe back instead of 16 + 4), then shf_use_uid_parts() +
 * shf_put_key_val() per key in window order; the store (files, uids) ends as
 * shf_put_batch_var() leaves it. perm_out / uids_out (optional, n entries):
 * the order used and shf_uid after each put (in batch index order). Returns as
 * shf_put_batch_var_win_ordered(). */
static inline int64_t shf_put_batch_var_parts_win_ordered(SHF *shf, const char *bytes, const uint64_t *offsets,
                                                          uint64_t n, const char *vals, const uint64_t *val_offsets,
                                                          uint32_t *perm_out, uint32_t *uids_out)
{
    if (n == 0) return 0;
    uint64_t *parts = (uint64_t *)malloc(n * sizeof *parts);
    uint32_t *perm = perm_out ? perm_out : (uint32_t *)malloc(n * sizeof *perm);
    if (!parts || !perm) {
        free(parts);
        if (!perm_out) free(perm);
        return SHF_HB_ERR_NOMEM;
    }
    int rc = shf_uid_parts_batch_var_win(bytes, offsets, n, SHF_HASH_BATCH_SEED, parts, perm, NULL, SHF_HASH_MEM_HOST);
    uint64_t j = 0;
    if (rc == SHF_HB_OK)
        for (; j < n; ++j) {
            const uint64_t i = perm[j];
            shf_use_uid_parts(bytes + offsets[i], (uint32_t)(offsets[i + 1] - offsets[i]), parts[i]);
            if (shf_put_key_val(shf, vals + val_offsets[i], (uint32_t)(val_offsets[i + 1] - val_offsets[i])) !=
                SHF_RET_KEY_PUT)
                break;
            if (uids_out) uids_out[i] = shf_uid;
        }
    free(parts);
    if (!perm_out) free(perm);
    return rc == SHF_HB_OK ? (int64_t)j : rc;
}

/* Get n keys with their batch hashes in window order (perm from shf_win_order
 * of those hashes): shf_get_key_val_copy() per key, on_found(ctx, i) with the
 * key's batch index i for every key found (shf_val / shf_val_len hold its
 * value then). Returns the keys found. */
static inline uint64_t shf_get_batch_win_ordered(SHF *shf, const char *bytes, const uint64_t *offsets, uint64_t n,
                                                 const shf_hash128 *hashes, const uint32_t *perm,
                                                 void (*on_found)(void *ctx, uint64_t i), void *ctx)
{
    uint64_t found = 0;
    for (uint64_t j = 0; j < n; ++j) {
        const uint64_t i = perm[j];
        shf_use_hash(bytes + offsets[i], (uint32_t)(offsets[i + 1] - offsets[i]), &hashes[i]);
        if (shf_get_key_val_copy(shf) == SHF_RET_KEY_FOUND) {
            ++found;
            if (on_found) on_found(ctx, i);
        }
    }
    return found;
}

/* One worker's share of a window-ordered batch: the puts of the keys of
 * windows [win_lo, win_hi) (perm and win_start from shf_win_order of the
 * batch's hashes), in order. Workers -- processes, each with its own
 * shf_attach() handle -- that take disjoint window ranges never share a
 * window's lock or structures (put 3.7x faster on 16 workers than slices of
 * the batch), and the store ends as a single batch-order
 * put leaves it, up to the uids tabs get when workers' parts interleave.
 * Returns the keys put (win_start[win_hi] - win_start[win_lo] when all went
 * in, else the count before the first put that did not return
 * SHF_RET_KEY_PUT), or SHF_HB_ERR_ARG for a bad range. */
static inline int64_t shf_put_batch_win_range(SHF *shf, const char *bytes, const uint64_t *offsets,
                                              const shf_hash128 *hashes, const uint32_t *perm,
                                              const uint32_t *win_start, uint32_t win_lo, uint32_t win_hi,
                                              const char *vals, const uint64_t *val_offsets)
{
    if (win_lo > win_hi || win_hi > 256) return SHF_HB_ERR_ARG;
    int64_t put = 0;
    for (uint64_t j = win_start[win_lo]; j < win_start[win_hi]; ++j, ++put) {
        const uint64_t i = perm[j];
        shf_use_hash(bytes + offsets[i], (uint32_t)(offsets[i + 1] - offsets[i]), &hashes[i]);
        if (shf_put_key_val(shf, vals + val_offsets[i], (uint32_t)(val_offsets[i + 1] - val_offsets[i])) !=
            SHF_RET_KEY_PUT)
            break;
    }
    return put;
}

#endif /* SHF_HASH_BATCH_SHF_H */
