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
#include <sys/wait.h>
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

/* ---- f4: shf_tab_part() / shf_tab_shrink() captured from the reference ------
 * Puts keys [0, n) one by one with the reference's own shf_make_hash() +
 * shf_put_key_val() (value: the key index, 8 bytes; in a fixed-length store
 * fixed_val_len bytes of it, repeated). Before every put it reads the key's
 * row from its tab file: a put into a full row parts that tab (shf.c:829-834 ->
 * shf_tab_part() at :722-779, which ends in shf_tab_shrink() at :678-720).
 * For up to max_caps such puts (and only those that parted exactly once) it
 * writes into out_dir:
 *   cap<c>.before  tab_old's file before the put
 *   cap<c>.old     tab_old's file after the put (re-created by the shrink)
 *   cap<c>.new     tab_new's file after the put
 *   cap<c>.meta    u32 {win, tab_old, tab_new, shf_uid of the put, key index,
 *                  fixed, fixed_key_len, fixed_val_len, data_needed_factor},
 *                  then the window's 2048 u16 tab2 -> tab map before and after.
 * fixed_key_len > 0 makes a fixed-length store (shf_set_is_fixed_len); the
 * data-needed factor is the reference's tab growth factor (shf.c:565).
 * Returns the number of captures, or < 0 (-3 store, -4 I/O). */
static int ref_copy_file(const char *from, const char *to)
{
    const int in = open(from, O_RDONLY);
    if (in < 0) return -1;
    const int out = open(to, O_WRONLY | O_CREAT | O_TRUNC, 0600);
    if (out < 0) { close(in); return -1; }
    char buf[1 << 16];
    ssize_t got;
    int rc = 0;
    while ((got = read(in, buf, sizeof buf)) > 0)
        if (write(out, buf, (size_t)got) != got) { rc = -1; break; }
    if (got < 0) rc = -1;
    close(in);
    close(out);
    return rc;
}

int64_t ref_part_capture(const char *folder, const char *name, const uint8_t *bytes, const uint64_t *offsets,
                         uint64_t n, uint32_t fixed_key_len, uint32_t fixed_val_len, uint32_t factor,
                         uint32_t max_caps, const char *out_dir)
{
    shf_init();
    SHF *shf = shf_attach(folder, name, 0);
    if (!shf) return -3;
    shf_set_is_lockable(shf, 0);
    if (fixed_key_len) shf_set_is_fixed_len(shf, fixed_key_len, fixed_val_len);
    shf_set_data_need_factor(factor ? factor : 1);
    char val[4096];
    int64_t caps = 0;
    for (uint64_t i = 0; i < n && caps < (int64_t)max_caps; ++i) {
        const char *key = (const char *)bytes + offsets[i];
        const uint32_t key_len = (uint32_t)(offsets[i + 1] - offsets[i]);
        uint32_t val_len = sizeof(i);
        if (fixed_key_len) {
            val_len = fixed_val_len;
            for (uint32_t b = 0; b < val_len && b < sizeof val; ++b) val[b] = ((const char *)&i)[b % sizeof(i)];
        } else {
            memcpy(val, &i, sizeof(i));
        }
        shf_make_hash(key, key_len);
        const uint32_t win = shf_hash.u16[0] % SHF_WINS_PER_SHF;
        const uint32_t tab2 = shf_hash.u16[1] % SHF_TABS_PER_WIN;
        const uint32_t row = shf_hash.u16[2] % SHF_ROWS_PER_TAB;
        volatile SHF_WIN_MMAP *w = &shf->shf_mmap->wins[win];
        const uint32_t tab_old = w->tabs[tab2].tab;
        const uint32_t used0 = w->tabs_used;
        char file_old[512];
        snprintf(file_old, sizeof file_old, "%s/%s.shf/%03u/%04u.tab", shf->path, shf->name, win, tab_old);
        SHF_ROW_MMAP r;
        int full = 0;
        {
            const int fd = open(file_old, O_RDONLY);
            if (fd < 0) { (void)shf_del(shf); return -4; }
            const ssize_t got = pread(fd, &r, sizeof r, offsetof(SHF_TAB_MMAP, row) + row * sizeof r);
            close(fd);
            if (got != (ssize_t)sizeof r) { (void)shf_del(shf); return -4; }
            full = 1;
            for (uint32_t k = 0; k < SHF_REFS_PER_ROW; ++k) full &= r.ref[k].pos != 0;
        }
        char path[1024];
        uint16_t map_before[SHF_TABS_PER_WIN];
        if (full) {
            for (uint32_t t2 = 0; t2 < SHF_TABS_PER_WIN; ++t2) map_before[t2] = w->tabs[t2].tab;
            snprintf(path, sizeof path, "%s/cap%lld.before", out_dir, (long long)caps);
            if (ref_copy_file(file_old, path)) { (void)shf_del(shf); return -4; }
        }
        if (shf_put_key_val(shf, val, val_len) != SHF_RET_KEY_PUT) { (void)shf_del(shf); return -3; }
        if (!full || w->tabs_used != used0 + 1) continue;  /* no part, or more than one */
        const uint32_t tab_new = used0;
        char file_new[512];
        snprintf(file_new, sizeof file_new, "%s/%s.shf/%03u/%04u.tab", shf->path, shf->name, win, tab_new);
        snprintf(path, sizeof path, "%s/cap%lld.old", out_dir, (long long)caps);
        if (ref_copy_file(file_old, path)) { (void)shf_del(shf); return -4; }
        snprintf(path, sizeof path, "%s/cap%lld.new", out_dir, (long long)caps);
        if (ref_copy_file(file_new, path)) { (void)shf_del(shf); return -4; }
        uint32_t meta[9] = {win, tab_old, tab_new, shf_uid, (uint32_t)i, fixed_key_len ? 1u : 0u, fixed_key_len,
                            fixed_val_len, factor ? factor : 1u};
        uint16_t map_after[SHF_TABS_PER_WIN];
        for (uint32_t t2 = 0; t2 < SHF_TABS_PER_WIN; ++t2) map_after[t2] = w->tabs[t2].tab;
        snprintf(path, sizeof path, "%s/cap%lld.meta", out_dir, (long long)caps);
        const int fd = open(path, O_WRONLY | O_CREAT | O_TRUNC, 0600);
        if (fd < 0) { (void)shf_del(shf); return -4; }
        const int ok = write(fd, meta, sizeof meta) == (ssize_t)sizeof meta &&
                       write(fd, map_before, sizeof map_before) == (ssize_t)sizeof map_before &&
                       write(fd, map_after, sizeof map_after) == (ssize_t)sizeof map_after;
        close(fd);
        if (!ok) { (void)shf_del(shf); return -4; }
        ++caps;
    }
    shf_set_data_need_factor(1);
    (void)shf_del(shf);
    return caps;
}

/* ---- window order (shf_win_order): one batch put in a given order ---------
 * Keys order[0..n) (key i = bytes[offsets[i] .. offsets[i+1]), value: i as 8
 * bytes) are put with the supplied hashes (2 x u64 per key, the seam of
 * test.9.shf.c:176-182) into a fresh store folder/name; uids[i] = the shf_uid
 * the put of key i left (shf.c:852). Then every key is read back in the same
 * order (shf_get_key_val_copy) and checked. The store is detached, not
 * deleted: its files stay for the caller to compare. put_seconds /
 * get_seconds: the two loops' wall time. Returns the keys found with their
 * value (n when all went in), or < 0 (-1: store, -2: a put failed). */
int64_t ref_put_in_order(const char *folder, const char *name, const uint8_t *bytes, const uint64_t *offsets,
                         uint64_t n, const uint64_t *hashes, const uint32_t *order, uint32_t *uids, int lockable,
                         double *put_seconds, double *get_seconds)
{
    shf_init();
    SHF *shf = shf_attach(folder, name, 0);
    if (!shf) return -1;
    shf_set_is_lockable(shf, (uint32_t)lockable);
    double t0 = ref_now();
    for (uint64_t j = 0; j < n; ++j) {
        const uint64_t i = order ? order[j] : j;
        shf_hash.u64[0] = hashes[2 * i];
        shf_hash.u64[1] = hashes[2 * i + 1];
        shf_hash_key = (const char *)bytes + offsets[i];
        shf_hash_key_len = (uint32_t)(offsets[i + 1] - offsets[i]);
        if (shf_put_key_val(shf, (const char *)&i, sizeof(i)) != SHF_RET_KEY_PUT) {
            shf_detach(shf);
            return -2;
        }
        uids[i] = shf_uid;
    }
    double t1 = ref_now();
    int64_t good = 0;
    for (uint64_t j = 0; j < n; ++j) {
        const uint64_t i = order ? order[j] : j;
        shf_hash.u64[0] = hashes[2 * i];
        shf_hash.u64[1] = hashes[2 * i + 1];
        shf_hash_key = (const char *)bytes + offsets[i];
        shf_hash_key_len = (uint32_t)(offsets[i + 1] - offsets[i]);
        good += shf_get_key_val_copy(shf) == SHF_RET_KEY_FOUND && ref_val_is(i);
    }
    double t2 = ref_now();
    if (put_seconds) *put_seconds = t1 - t0;
    if (get_seconds) *get_seconds = t2 - t1;
    shf_detach(shf);
    return good;
}

/* ---- window order with processes: the reference's put/get loops on T processes --
 * (The reference's lock is a process-level lock: several handles in one
 * process are not a supported use, so the workers are forked processes, as in
 * the reference's own multi-process tests.) Worker t attaches its own handle
 * to store folder/name (created here first) and runs keys idx[starts[t] ..
 * starts[t+1]) (idx NULL: batch order) through shf_put_key_val (value: the key
 * index); after every worker's puts, the same keys through
 * shf_get_key_val_copy, checking each value. With idx = the window order and
 * starts at window boundaries (shf_win_order's win_start), the workers'
 * windows are disjoint: no window lock or window structure is shared. The
 * caller must not have started threads the children need (call it from a
 * process that has not touched the GPU). Returns the keys found with their
 * value, or < 0. */
static int64_t ref_worker(const char *folder, const char *name, const uint8_t *bytes, const uint64_t *offsets,
                          const uint64_t *hashes, const uint32_t *idx, uint64_t lo, uint64_t hi, int lockable, int op)
{
    SHF *shf = shf_attach(folder, name, 0);
    if (!shf) return -1;
    shf_set_is_lockable(shf, (uint32_t)lockable);
    int64_t good = 0;
    for (uint64_t j = lo; j < hi; ++j) {
        const uint64_t i = idx ? idx[j] : j;
        shf_hash.u64[0] = hashes[2 * i];
        shf_hash.u64[1] = hashes[2 * i + 1];
        shf_hash_key = (const char *)bytes + offsets[i];
        shf_hash_key_len = (uint32_t)(offsets[i + 1] - offsets[i]);
        if (op == 0) good += shf_put_key_val(shf, (const char *)&i, sizeof(i)) == SHF_RET_KEY_PUT;
        else good += shf_get_key_val_copy(shf) == SHF_RET_KEY_FOUND && ref_val_is(i);
    }
    shf_detach(shf);
    return good;
}

int64_t ref_put_get_procs(const char *folder, const char *name, const uint8_t *bytes, const uint64_t *offsets,
                          const uint64_t *hashes, const uint32_t *idx, const uint64_t *starts, int nprocs,
                          int lockable, double *put_seconds, double *get_seconds)
{
    if (nprocs < 1 || nprocs > 256) return -1;
    shf_init();
    SHF *shf = shf_attach(folder, name, 0);
    if (!shf) return -1;
    int64_t *res = mmap(NULL, 256 * sizeof(int64_t), PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
    if (res == MAP_FAILED) return -2;
    int64_t found = 0;
    for (int op = 0; op < 2; ++op) {
        const double t0 = ref_now();
        pid_t pids[256];
        for (int t = 0; t < nprocs; ++t) {
            pids[t] = fork();
            if (pids[t] == 0) {
                res[t] = ref_worker(folder, name, bytes, offsets, hashes, idx, starts[t], starts[t + 1], lockable, op);
                _exit(0);
            }
            if (pids[t] < 0) return -2;
        }
        int64_t good = 0;
        for (int t = 0; t < nprocs; ++t) {
            int st = 0;
            waitpid(pids[t], &st, 0);
            good += res[t];
        }
        const double dt = ref_now() - t0;
        if (op == 0) {
            if (put_seconds) *put_seconds = dt;
            if (good != (int64_t)(starts[nprocs] - starts[0])) {
                munmap(res, 256 * sizeof(int64_t));
                shf_detach(shf);
                return -3;
            }
        } else {
            if (get_seconds) *get_seconds = dt;
            found = good;
        }
    }
    munmap(res, 256 * sizeof(int64_t));
    shf_detach(shf);
    return found;
}
