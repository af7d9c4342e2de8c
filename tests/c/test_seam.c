/*
 * The drop-in seam, proven from C (no ctypes): this program links
 * libshf_hash_batch.so (the product) with the reference's own table engine
 * (src/shf.c + src/murmurhash3.c, compiled by oracle/Makefile into oracle/_ref/)
 * and runs, on one store:
 *
 *   1. INTEGRATION.md §3's batched put loop: shf_put_batch_var() -- one GPU
 *      batch hash (shf_hash_batch_var, host memory), then shf_use_hash() +
 *      shf_put_key_val() per key (include/shf_hash_batch_shf.h);
 *   2. the reference's own get loop (shf_make_hash() + shf_get_key_val_copy(),
 *      test.9.shf.c:442-445 shape) over the stored keys and as many absent
 *      ones: every stored key found with its value, no absent key found;
 *   3. INTEGRATION.md §6's probed get loop: the store's rows exported into a
 *      row index, the whole batch hashed and probed on the GPU
 *      (shf_probe_batch_var, host memory), shf_get_batch_probed(): the same
 *      answers, most stored keys served by the uid path;
 *   4. fixed 16-byte keys: shf_hash_batch_fixed + shf_use_hash + put, then
 *      the reference's get with its CPU hash finds every one;
 *   5./6. the window-ordered put and window ranges;
 *   7. 8-B UID parts (shf_uid_parts_batch_var, host memory) through
 *      shf_use_uid_parts: a store put from parts is byte-equal to one put from
 *      the full hashes, with the same shf_uid per key, and the reference's
 *      own get finds every key in it; gets and dels with the parts in the seam
 *      give the reference's answers;
 *   8. the same put in the window order of the parts (shf_uid_parts_batch_var_win):
 *      again byte-equal, uids included.
 *
 * TEST INFRASTRUCTURE: built by tests/c/Makefile where /root/reference exists
 * (the reference's headers are needed to compile it), into tests/c/build/, which
 * travels to the GPU box with the tree. Exit status: 0 pass, 1 fail, 2 no usable
 * GPU (the library refused: no CPU fallback).
 */
#define _GNU_SOURCE
#include <ftw.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "shf.private.h"
#include "shf.h"
#include "shf_hash_batch_shf.h"

/* oracle/ref_export.c (test infrastructure): rows + tab map of a store */
extern int64_t ref_export_rows(SHF *shf, uint32_t *tab_slot, uint8_t *rows, uint64_t max_slots);

static uint64_t splitmix(uint64_t *s)
{
    uint64_t z = (*s += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

static int fail(const char *what)
{
    fprintf(stderr, "test_seam: FAIL: %s\n", what);
    return 1;
}

static int remove_entry(const char *path, const struct stat *sb, int flag, struct FTW *ftw)
{
    (void)sb;
    (void)flag;
    (void)ftw;
    return remove(path);
}

/* Every tab file of store `a` byte-equal to the same file of store `b` (both in folder),
 * with the same tab counts per window; the number of files compared, or -1. */
static int64_t same_store_files(const char *folder, const char *a, SHF *sa, const char *b, SHF *sb)
{
    int64_t same = 0;
    for (uint32_t win = 0; win < SHF_WINS_PER_SHF; ++win) {
        if (sa->shf_mmap->wins[win].tabs_used != sb->shf_mmap->wins[win].tabs_used) return -1;
        for (uint32_t tab = 0; tab < sa->shf_mmap->wins[win].tabs_used; ++tab) {
            char pa[512], pb[512];
            snprintf(pa, sizeof pa, "%s/%s.shf/%03u/%04u.tab", folder, a, win, tab);
            snprintf(pb, sizeof pb, "%s/%s.shf/%03u/%04u.tab", folder, b, win, tab);
            FILE *fa = fopen(pa, "rb"), *fb = fopen(pb, "rb");
            if (!fa || !fb) {
                if (fa) fclose(fa);
                if (fb) fclose(fb);
                return -1;
            }
            int ca, cb;
            do {
                ca = fgetc(fa);
                cb = fgetc(fb);
            } while (ca == cb && ca != EOF);
            fclose(fa);
            fclose(fb);
            if (ca != cb) return -1;
            ++same;
        }
    }
    return same;
}

/* The UID-parts word of a full hash (shf_hash_batch.h SHF_UID_PARTS_*). */
static uint64_t parts_of(const shf_hash128 *h)
{
    return (h->h1 & 0xff) | ((h->h1 >> 16) & 0x7ff) << 8 | ((h->h1 >> 32) & 0x1ff) << 19 |
           (h->h2 & 0x1fffff) << 32;
}

static uint64_t good_values;
static void check_value(void *ctx, uint64_t i)
{
    (void)ctx;
    good_values += shf_val_len == sizeof(i) && memcmp(shf_val, &i, sizeof(i)) == 0;
}

int main(int argc, char **argv)
{
    const uint64_t n_put = argc > 1 ? strtoull(argv[1], 0, 10) : 200000, n_absent = n_put / 10;
    const uint64_t n = n_put + n_absent;
    const int rc0 = shf_hash_batch_check_device();
    if (rc0 != SHF_HB_OK) {
        fprintf(stderr, "test_seam: no usable GPU: %s\n", shf_hash_batch_strerror(rc0));
        return 2;
    }

    /* keys 4..67 bytes, unique (the key index in their first 4-8 bytes), values = the key index (8 bytes) */
    uint64_t *off = malloc((n + 1) * sizeof *off), *voff = malloc((n + 1) * sizeof *voff);
    uint64_t st = 0x5348460000000077ull;
    off[0] = voff[0] = 0;
    for (uint64_t i = 0; i < n; ++i) {
        off[i + 1] = off[i] + 4 + splitmix(&st) % 64;
        voff[i + 1] = voff[i] + 8;
    }
    char *bytes = malloc(off[n] + 8), *vals = malloc(8 * n);
    for (uint64_t b = 0; b < off[n]; b += 8) {
        const uint64_t v = splitmix(&st);
        memcpy(bytes + b, &v, 8);
    }
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t len = off[i + 1] - off[i];
        memcpy(bytes + off[i], &i, len < 8 ? len : 8);
        memcpy(vals + 8 * i, &i, 8);
    }
    char folder[] = "/dev/shm/seamXXXXXX";
    if (!mkdtemp(folder)) return fail("mkdtemp");
    shf_init();
    SHF *shf = shf_attach(folder, "seam", 0);
    if (!shf) return fail("shf_attach");

    /* 1. batched put with GPU hashes */
    const int64_t put = shf_put_batch_var(shf, bytes, off, n_put, vals, voff);
    if (put != (int64_t)n_put) {
        fprintf(stderr, "put %lld of %llu\n", (long long)put, (unsigned long long)n_put);
        return fail("shf_put_batch_var");
    }

    /* 2. the reference's own get (CPU hash): the answer of record, per key */
    uint8_t *want_found = calloc(n, 1);
    uint64_t *want_val = calloc(n, sizeof *want_val);
    uint64_t ref_found = 0, ref_right = 0;
    for (uint64_t i = 0; i < n; ++i) {
        shf_make_hash(bytes + off[i], (uint32_t)(off[i + 1] - off[i]));
        if (shf_get_key_val_copy(shf) == SHF_RET_KEY_FOUND) {
            want_found[i] = 1;
            memcpy(&want_val[i], shf_val, 8);
            ++ref_found;
            ref_right += i < n_put && want_val[i] == i;
        }
    }
    /* every stored key found with its own value, no absent key found */
    if (ref_right != n_put || ref_found != n_put) return fail("reference get after GPU-hashed put");

    /* 3. probed get: export, index, probe on the GPU, the §6 loop */
    const uint64_t max_slots = 4096;
    uint32_t *tab_slot = malloc(SHF_ROW_INDEX_TABS * sizeof *tab_slot);
    uint8_t *rows = malloc(max_slots * SHF_ROW_INDEX_SLOT_BYTES);
    const int64_t slots = ref_export_rows(shf, tab_slot, rows, max_slots);
    if (slots <= 0) return fail("ref_export_rows");
    shf_row_index *ix = NULL;
    if (shf_row_index_create((uint64_t)slots, &ix) != SHF_HB_OK) return fail("shf_row_index_create");
    if (shf_row_index_set_tabs(ix, tab_slot) != SHF_HB_OK) return fail("set_tabs");
    if (shf_row_index_set_rows(ix, 0, (uint64_t)slots, rows) != SHF_HB_OK) return fail("set_rows");
    shf_hash128 *h = malloc(n * sizeof *h);
    shf_probe *pr = malloc(n * sizeof *pr);
    if (shf_probe_batch_var(ix, bytes, off, n, SHF_HASH_BATCH_SEED, h, pr, SHF_HASH_MEM_HOST) != SHF_HB_OK)
        return fail("shf_probe_batch_var");
    uint64_t fast = 0;
    good_values = 0;
    const uint64_t found = shf_get_batch_probed(shf, bytes, off, n, h, pr, check_value, NULL, &fast);
    /* the probed loop must give the reference's answers: same found count, every stored key's value */
    if (found != ref_found) return fail("probed get: found count differs from the reference's get");
    if (good_values != ref_right) return fail("probed get: values differ from the reference's get");
    if (fast < n_put / 2) return fail("probed get: uid path unused");
    /* GPU hash == CPU shf_make_hash for every key */
    for (uint64_t i = 0; i < n; ++i) {
        shf_make_hash(bytes + off[i], (uint32_t)(off[i + 1] - off[i]));
        if (shf_hash.u64[0] != h[i].h1 || shf_hash.u64[1] != h[i].h2) return fail("GPU hash != shf_make_hash");
    }
    shf_row_index_destroy(ix);

    /* 4. fixed 16-byte keys */
    const uint64_t nf = 50000;
    char *fk = malloc(16 * nf);
    for (uint64_t i = 0; i < 2 * nf; ++i) {
        const uint64_t v = splitmix(&st);
        memcpy(fk + 8 * i, &v, 8);
    }
    for (uint64_t i = 0; i < nf; ++i) memcpy(fk + 16 * i, &i, 8);
    shf_hash128 *fh = malloc(nf * sizeof *fh);
    if (shf_hash_batch_fixed(fk, 16, nf, SHF_HASH_BATCH_SEED, fh, SHF_HASH_MEM_HOST) != SHF_HB_OK)
        return fail("shf_hash_batch_fixed");
    char fshf_name[] = "seamfixed";
    SHF *fshf = shf_attach(folder, fshf_name, 0);
    if (!fshf) return fail("shf_attach fixed");
    for (uint64_t i = 0; i < nf; ++i) {
        shf_use_hash(fk + 16 * i, 16, &fh[i]);
        if (shf_put_key_val(fshf, (const char *)&i, 8) != SHF_RET_KEY_PUT) return fail("fixed put");
    }
    uint64_t ffound = 0;
    for (uint64_t i = 0; i < nf; ++i) {
        shf_make_hash(fk + 16 * i, 16);
        ffound += shf_get_key_val_copy(fshf) == SHF_RET_KEY_FOUND && memcmp(shf_val, &i, 8) == 0;
    }
    if (ffound != nf) return fail("fixed keys: reference get after GPU-hashed put");

    /* 5. the same batch put in the GPU's window order into a second store:
     *    identical uids (the put loop leaves shf_uid) and every tab file equal */
    SHF *wshf = shf_attach(folder, "seamwin", 0);
    if (!wshf) return fail("shf_attach window order");
    uint32_t *perm = malloc(n_put * sizeof *perm);
    if (shf_put_batch_var_win_ordered(wshf, bytes, off, n_put, vals, voff, perm) != (int64_t)n_put)
        return fail("shf_put_batch_var_win_ordered");
    for (uint64_t j = 1; j < n_put; ++j) /* windows ascending, batch order inside each */
        if ((h[perm[j]].h1 & 0xff) < (h[perm[j - 1]].h1 & 0xff) ||
            ((h[perm[j]].h1 & 0xff) == (h[perm[j - 1]].h1 & 0xff) && perm[j] < perm[j - 1]))
            return fail("window order: not a stable sort by window");
    const int64_t same_files = same_store_files(folder, "seam", shf, "seamwin", wshf);
    if (same_files < 0) return fail("window order: tab files differ");
    /* a get batch (stored and absent keys) in window order gives the reference's answers */
    shf_hash128 *hw = malloc(n * sizeof *hw);
    uint32_t *permq = malloc(n * sizeof *permq);
    memcpy(hw, h, n * sizeof *hw);
    if (shf_win_order(hw, n, permq, NULL, SHF_HASH_MEM_HOST) != SHF_HB_OK) return fail("shf_win_order");
    good_values = 0;
    const uint64_t wfound2 = shf_get_batch_win_ordered(wshf, bytes, off, n, h, permq, check_value, NULL);
    if (wfound2 != ref_found || good_values != ref_right) return fail("window-ordered get: answers differ");

    /* 6. window ranges: 4 workers, each its own handle on a third store, each putting windows
     *    [64 w, 64 w + 64) of the same order (one after another here: this process has touched the
     *    GPU, so it forks nothing; tools/win_order_procs.py times the ranges on forked workers) */
    uint32_t *ws = malloc(257 * sizeof *ws);
    if (shf_win_order(h, n_put, perm, ws, SHF_HASH_MEM_HOST) != SHF_HB_OK) return fail("shf_win_order ranges");
    int64_t range_put = 0;
    for (uint32_t w = 0; w < 4; ++w) {
        SHF *mine = shf_attach(folder, "seamrange", 0);
        if (!mine) return fail("shf_attach ranges");
        range_put += shf_put_batch_win_range(mine, bytes, off, h, perm, ws, 64 * w, 64 * w + 64, vals, voff);
        shf_detach(mine);
    }
    if (shf_put_batch_win_range(shf, bytes, off, h, perm, ws, 3, 2, vals, voff) != SHF_HB_ERR_ARG)
        return fail("window ranges: bad range accepted");
    SHF *rshf = shf_attach(folder, "seamrange", 0);
    if (!rshf) return fail("shf_attach ranges");
    if (range_put != (int64_t)n_put) return fail("window ranges: puts");
    good_values = 0;
    const uint64_t rfound = shf_get_batch_win_ordered(rshf, bytes, off, n, h, permq, check_value, NULL);
    if (rfound != ref_found || good_values != ref_right) return fail("window ranges: get answers differ");
    shf_detach(rshf);

    /* 7. UID parts (8 B per key from the GPU) through shf_use_uid_parts: a store put from
     *    parts ends byte for byte as one put from the full hashes, with the same shf_uid per
     *    key, and the reference's own get (CPU shf_make_hash) finds every key in it */
    uint64_t *parts = malloc(n * sizeof *parts);
    if (shf_uid_parts_batch_var(bytes, off, n, SHF_HASH_BATCH_SEED, parts, SHF_HASH_MEM_HOST) != SHF_HB_OK)
        return fail("shf_uid_parts_batch_var");
    for (uint64_t i = 0; i < n; ++i)
        if (parts[i] != parts_of(&h[i])) return fail("UID parts != the parts of the GPU hash");
    SHF *hshf = shf_attach(folder, "seamuidh", 0);
    SHF *pshf = shf_attach(folder, "seamuidp", 0);
    if (!hshf || !pshf) return fail("shf_attach uid parts");
    uint32_t *uid_h = malloc(n_put * sizeof *uid_h), *uid_p = malloc(n_put * sizeof *uid_p);
    for (uint64_t i = 0; i < n_put; ++i) {
        shf_use_hash(bytes + off[i], (uint32_t)(off[i + 1] - off[i]), &h[i]);
        if (shf_put_key_val(hshf, vals + voff[i], 8) != SHF_RET_KEY_PUT) return fail("uid parts: full-hash put");
        uid_h[i] = shf_uid;
    }
    if (shf_put_batch_var_parts(pshf, bytes, off, n_put, vals, voff, uid_p) != (int64_t)n_put)
        return fail("shf_put_batch_var_parts");
    uint64_t uid_same = 0;
    for (uint64_t i = 0; i < n_put; ++i) uid_same += uid_h[i] == uid_p[i] && uid_p[i] != SHF_UID_NONE;
    if (uid_same != n_put) return fail("uid parts: shf_uid differs from the full-hash put");
    const int64_t parts_same_files = same_store_files(folder, "seamuidh", hshf, "seamuidp", pshf);
    if (parts_same_files < 0) return fail("uid parts: tab files differ from the full-hash put");
    uint64_t pfound = 0, pright = 0;
    for (uint64_t i = 0; i < n; ++i) {  /* the reference's own get, CPU hash */
        shf_make_hash(bytes + off[i], (uint32_t)(off[i + 1] - off[i]));
        if (shf_get_key_val_copy(pshf) == SHF_RET_KEY_FOUND) {
            ++pfound;
            pright += i < n_put && shf_val_len == 8 && memcmp(shf_val, &i, 8) == 0;
        }
    }
    if (pfound != n_put || pright != n_put) return fail("uid parts: reference get after a parts put");
    /* and a get with the parts in the seam gives the reference's answers too */
    uint64_t pgot = 0, pgot_any = 0;
    for (uint64_t i = 0; i < n; ++i) {
        shf_use_uid_parts(bytes + off[i], (uint32_t)(off[i + 1] - off[i]), parts[i]);
        if (shf_get_key_val_copy(pshf) == SHF_RET_KEY_FOUND) {
            ++pgot_any;
            pgot += i < n_put && shf_val_len == 8 && memcmp(shf_val, &i, 8) == 0;
        }
    }
    if (pgot != n_put || pgot_any != n_put) return fail("uid parts: get through shf_use_uid_parts");
    /* del through the parts (shf_del_key_val finds the key with the same bits): every even key gone,
     * every odd one still found by the reference's own get; deleting an absent key finds nothing */
    uint64_t pdel = 0, pdel_absent = 0;
    for (uint64_t i = 0; i < n; i += 2) {
        shf_use_uid_parts(bytes + off[i], (uint32_t)(off[i + 1] - off[i]), parts[i]);
        const uint32_t r = shf_del_key_val(pshf);
        if (i < n_put) pdel += r == SHF_RET_KEY_FOUND;
        else pdel_absent += r == SHF_RET_KEY_FOUND;
    }
    uint64_t pleft = 0, pleft_right = 0;
    for (uint64_t i = 0; i < n; ++i) {
        shf_make_hash(bytes + off[i], (uint32_t)(off[i + 1] - off[i]));
        if (shf_get_key_val_copy(pshf) == SHF_RET_KEY_FOUND) {
            ++pleft;
            pleft_right += (i & 1) && i < n_put && memcmp(shf_val, &i, 8) == 0;
        }
    }
    if (pdel != (n_put + 1) / 2 || pdel_absent != 0 || pleft != n_put / 2 || pleft_right != n_put / 2)
        return fail("uid parts: del through shf_use_uid_parts");
    /* fixed 16-byte keys: the parts of the fixed-length entry point */
    uint64_t *fparts = malloc(nf * sizeof *fparts);
    if (shf_uid_parts_batch_fixed(fk, 16, nf, SHF_HASH_BATCH_SEED, fparts, SHF_HASH_MEM_HOST) != SHF_HB_OK)
        return fail("shf_uid_parts_batch_fixed");
    for (uint64_t i = 0; i < nf; ++i)
        if (fparts[i] != parts_of(&fh[i])) return fail("fixed UID parts != the parts of the GPU hash");
    /* 8. the window-ordered put from UID parts (shf_put_batch_var_parts_win_ordered): a stable order
     *    by the parts' window, and the store byte-equal, uids included, to the full-hash put */
    SHF *oshf = shf_attach(folder, "seamuidwin", 0);
    if (!oshf) return fail("shf_attach uid parts window order");
    uint32_t *operm = malloc(n_put * sizeof *operm), *ouid = malloc(n_put * sizeof *ouid);
    if (shf_put_batch_var_parts_win_ordered(oshf, bytes, off, n_put, vals, voff, operm, ouid) != (int64_t)n_put)
        return fail("shf_put_batch_var_parts_win_ordered");
    for (uint64_t j = 1; j < n_put; ++j)
        if ((parts[operm[j]] & 0xff) < (parts[operm[j - 1]] & 0xff) ||
            ((parts[operm[j]] & 0xff) == (parts[operm[j - 1]] & 0xff) && operm[j] < operm[j - 1]))
            return fail("uid parts window order: not a stable sort by window");
    uint64_t ouid_same = 0;
    for (uint64_t i = 0; i < n_put; ++i) ouid_same += ouid[i] == uid_h[i];
    if (ouid_same != n_put) return fail("uid parts window order: shf_uid differs from the full-hash put");
    const int64_t owin_same_files = same_store_files(folder, "seamuidh", hshf, "seamuidwin", oshf);
    if (owin_same_files < 0) return fail("uid parts window order: tab files differ from the full-hash put");
    shf_detach(oshf);
    shf_detach(hshf);
    shf_detach(pshf);

    printf("{\"n_put\": %llu, \"n_query\": %llu, \"ref_found\": %llu, \"ref_right\": %llu, \"probed_found\": %llu, "
           "\"probed_fast\": %llu, \"slots\": %lld, \"fixed_found\": %llu, \"win_order_same_tab_files\": %lld, "
           "\"win_order_found\": %llu, \"win_range_put\": %lld, \"parts_same_uids\": %llu, "
           "\"parts_same_tab_files\": %lld, \"parts_ref_found\": %llu, \"parts_get_found\": %llu, "
           "\"parts_deleted\": %llu, \"parts_left\": %llu, \"parts_win_same_uids\": %llu, "
           "\"parts_win_same_tab_files\": %lld}\n",
           (unsigned long long)n_put, (unsigned long long)n, (unsigned long long)ref_found,
           (unsigned long long)ref_right, (unsigned long long)found, (unsigned long long)fast, (long long)slots,
           (unsigned long long)ffound, (long long)same_files, (unsigned long long)wfound2,
           (long long)range_put, (unsigned long long)uid_same, (long long)parts_same_files,
           (unsigned long long)pright, (unsigned long long)pgot, (unsigned long long)pdel,
           (unsigned long long)pleft, (unsigned long long)ouid_same, (long long)owin_same_files);
    shf_detach(wshf);
    /* the stores' files go with the folder (shf_del would run `du` and `rm` through popen) */
    shf_detach(shf);
    shf_detach(fshf);
    nftw(folder, remove_entry, 16, FTW_DEPTH | FTW_PHYS);
    return 0;
}
