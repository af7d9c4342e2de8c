/*
 * TEST INFRASTRUCTURE ONLY -- compiled (by oracle/Makefile) against the
 * REFERENCE's own headers where they lie (/root/reference/src) and linked into
 * oracle/_ref/libref_shf.so with its shf.c. Never committed as a binary, never
 * part of the product.
 *
 * Purpose: pin the row pre-probe to the reference itself.
 * A store is filled and queried by the reference's own put/get, and its rows
 * are exported in the row-index layout of include/shf_hash_batch.h; the tests
 * then require the oracle (oracle_probe) and the GPU probe to agree with the
 * shf_uid the reference's get returned for every key.
 *
 * Reference structures used (src/shf.private.h):
 *   SHF (:156-171): shf_mmap, path, name
 *   SHF_WIN_MMAP (:84-96): tabs[2048].tab, tabs_used
 *   SHF_TAB_MMAP (:59-68): row[512] at offsetof(SHF_TAB_MMAP, row)
 *   tab files "<path>/<name>.shf/<win %03u>/<tab %04u>.tab" (src/shf.c:370, :488)
 */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <sys/types.h>
#include <time.h>
#include <unistd.h>

#include "shf.private.h"
#include "shf.h"

#define REF_SLOT_BYTES (SHF_ROWS_PER_TAB * SHF_SIZE_ROW) /* 65536 */

/* Export every tab's rows and the tab2 -> tab map of every window.
 *   tab_slot[(win << 11) | tab2] = (slot << 11) | tab
 *   rows[slot * 64 KiB ..]       = SHF_TAB_MMAP.row[] of (win, tab)
 * Slots are numbered window by window, tab by tab. The rows are read from the
 * tab files (the same pages the store's MAP_SHARED mappings hold), so the
 * export needs no tab to be mapped in this process.
 * Returns the number of slots, or < 0 (-1: more than max_slots, -2: I/O). */
int64_t ref_export_rows(SHF *shf, uint32_t *tab_slot, uint8_t *rows, uint64_t max_slots)
{
    _Static_assert(REF_SLOT_BYTES == 65536, "rows per tab");
    uint64_t slot = 0;
    for (uint32_t win = 0; win < SHF_WINS_PER_SHF; ++win) {
        volatile SHF_WIN_MMAP *w = &shf->shf_mmap->wins[win];
        const uint32_t used = w->tabs_used;
        const uint64_t first = slot;
        for (uint32_t tab = 0; tab < used; ++tab, ++slot) {
            if (slot >= max_slots) return -1;
            char file[512];
            snprintf(file, sizeof file, "%s/%s.shf/%03u/%04u.tab", shf->path, shf->name, win, tab);
            const int fd = open(file, O_RDONLY);
            if (fd < 0) return -2;
            const ssize_t got = pread(fd, rows + slot * REF_SLOT_BYTES, REF_SLOT_BYTES, offsetof(SHF_TAB_MMAP, row));
            close(fd);
            if (got != REF_SLOT_BYTES) return -2;
        }
        for (uint32_t tab2 = 0; tab2 < SHF_TABS_PER_WIN; ++tab2) {
            const uint32_t tab = w->tabs[tab2].tab;
            tab_slot[(win << 11) | tab2] = tab < used ? (uint32_t)((first + tab) << 11) | tab : 0xffffffffu;
        }
    }
    return (int64_t)slot;
}

/* Put keys [0, n_put) (value = the key's index, 8 B) with the reference's own
 * shf_make_hash() + shf_put_key_val(), then look up keys [0, n_query) with
 * shf_make_hash() + shf_get_key_val_addr() and record shf_uid (SHF_UID_NONE
 * when not found), then export the rows. Key i = bytes[offsets[i] ..
 * offsets[i+1]). Returns the slot count, or < 0 on failure (-3: store). */
int64_t ref_probe_fixture(const char *folder, const char *name, const uint8_t *bytes, const uint64_t *offsets,
                          uint64_t n_put, uint64_t n_query, uint32_t *uid_out, uint32_t *tab_slot, uint8_t *rows,
                          uint64_t max_slots)
{
    shf_init();
    SHF *shf = shf_attach(folder, name, 0);
    if (!shf) return -3;
    shf_set_is_lockable(shf, 0);
    for (uint64_t i = 0; i < n_put; ++i) {
        shf_make_hash((const char *)bytes + offsets[i], (uint32_t)(offsets[i + 1] - offsets[i]));
        if (shf_put_key_val(shf, (const char *)&i, sizeof(i)) != SHF_RET_KEY_PUT) {
            (void)shf_del(shf);
            return -3;
        }
    }
    for (uint64_t i = 0; i < n_query; ++i) {
        shf_make_hash((const char *)bytes + offsets[i], (uint32_t)(offsets[i + 1] - offsets[i]));
        uid_out[i] = shf_get_key_val_addr(shf) == SHF_RET_KEY_FOUND ? shf_uid : SHF_UID_NONE;
    }
    const int64_t slots = ref_export_rows(shf, tab_slot, rows, max_slots);
    (void)shf_del(shf);
    return slots;
}

/* ---- the f3 get loop, end to end, on the reference's own store ------------
 * A store that stays open across calls, so a test can export its rows, probe
 * them on the GPU, and feed the probe records back into the reference's get.
 * Values are the key index (8 bytes). */
SHF *ref_store_open(const char *folder, const char *name)
{
    shf_init();
    SHF *shf = shf_attach(folder, name, 0);
    if (shf) shf_set_is_lockable(shf, 0);
    return shf;
}

int64_t ref_store_put(SHF *shf, const uint8_t *bytes, const uint64_t *offsets, uint64_t n)
{
    for (uint64_t i = 0; i < n; ++i) {
        shf_make_hash((const char *)bytes + offsets[i], (uint32_t)(offsets[i + 1] - offsets[i]));
        if (shf_put_key_val(shf, (const char *)&i, sizeof(i)) != SHF_RET_KEY_PUT) return (int64_t)i;
    }
    return (int64_t)n;
}

void ref_store_close(SHF *shf) { (void)shf_del(shf); }

static double ref_now(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static int ref_val_is(uint64_t i) { return shf_val_len == sizeof(i) && memcmp(shf_val, &i, sizeof(i)) == 0; }

/* The reference's own get loop (test.9.shf.c:442-445 shape): shf_make_hash()
 * + shf_get_key_val_copy() per key. Returns keys found with the right value. */
int64_t ref_store_get_plain(SHF *shf, const uint8_t *bytes, const uint64_t *offsets, uint64_t n, double *seconds)
{
    int64_t good = 0;
    const double t0 = ref_now();
    for (uint64_t i = 0; i < n; ++i) {
        shf_make_hash((const char *)bytes + offsets[i], (uint32_t)(offsets[i + 1] - offsets[i]));
        good += shf_get_key_val_copy(shf) == SHF_RET_KEY_FOUND && ref_val_is(i);
    }
    if (seconds) *seconds = ref_now() - t0;
    return good;
}

/* The get loop INTEGRATION.md §6 describes, driven by GPU probe records
 * (4 u32 per key: uid, pos, mask | tab << 16, slot) and GPU hashes:
 *   candidate -> shf_get_uid_val_copy(uid) (shf.c:1037; checks pos and tab,
 *                not the key) + compare the stored key (len at key - 4,
 *                then the bytes) -> done;
 *   otherwise  -> the ordinary get with the GPU hash in the thread-local
 *                seam (test.9.shf.c:176-182).
 * Returns keys found with the right value; *fast = keys served by the uid path. */
int64_t ref_store_get_probed(SHF *shf, const uint8_t *bytes, const uint64_t *offsets, uint64_t n,
                             const uint32_t *probe, const uint64_t *hashes, uint64_t *fast, double *seconds)
{
    int64_t good = 0;
    uint64_t f = 0;
    const double t0 = ref_now();
    for (uint64_t i = 0; i < n; ++i) {
        const char *k = (const char *)bytes + offsets[i];
        const uint32_t kl = (uint32_t)(offsets[i + 1] - offsets[i]);
        const uint32_t *p = probe + 4 * i;
        if ((p[2] & 0xffffu) && shf_get_uid_val_copy(shf, p[0]) == SHF_RET_KEY_FOUND) {
            uint32_t stored_len;
            memcpy(&stored_len, (const char *)shf_key_addr - sizeof(stored_len), sizeof(stored_len));
            if (stored_len == kl && memcmp(shf_key_addr, k, kl) == 0) {
                good += ref_val_is(i);
                ++f;
                continue;
            }
        }
        shf_hash.u64[0] = hashes[2 * i];
        shf_hash.u64[1] = hashes[2 * i + 1];
        shf_hash_key = k;
        shf_hash_key_len = kl;
        good += shf_get_key_val_copy(shf) == SHF_RET_KEY_FOUND && ref_val_is(i);
    }
    if (seconds) *seconds = ref_now() - t0;
    if (fast) *fast = f;
    return good;
}
