/*
 * TEST INFRASTRUCTURE ONLY -- a thin harness linked with the REFERENCE's own
 * murmurhash3.c + shf.c (compiled from /root/reference/src by oracle/Makefile
 * into oracle/_ref/libref_shf.so; never committed, never shipped in the
 * product). It lets tests/golden/make_golden.py read the reference's
 * thread-local result, and lets bench.py time the reference's shf_make_hash()
 * loop (cpu_baseline kind "reference").
 *
 * Reference symbols used (not redeclared from its headers, to keep the
 * reference headers out of this file):
 *   void shf_make_hash(const char *key, uint32_t key_len);   src/shf.h:381
 *   __thread SHF_HASH shf_hash;   16-byte union, src/shf.private.h:180-187
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef struct { uint64_t u64[2]; } ref_hash16; /* same size/layout as SHF_HASH */

extern void shf_make_hash(const char *key, uint32_t key_len);
extern __thread ref_hash16 shf_hash;
extern void MurmurHash3_x64_128(const void *key, const int len, const uint32_t seed, void *out);

/* shf_make_hash() then copy the thread-local shf_hash out. */
void ref_make_hash_into(const char *key, uint32_t key_len, uint64_t out[2])
{
    shf_make_hash(key, key_len);
    out[0] = shf_hash.u64[0];
    out[1] = shf_hash.u64[1];
}

/* MurmurHash3_x64_128 directly (any seed). */
void ref_murmur3_into(const void *key, int len, uint32_t seed, uint64_t out[2])
{
    MurmurHash3_x64_128(key, len, seed, out);
}

void ref_hash_var(const uint8_t *bytes, const uint64_t *offsets, uint64_t n, uint64_t *out)
{
    for (uint64_t i = 0; i < n; ++i)
        ref_make_hash_into((const char *)bytes + offsets[i], (uint32_t)(offsets[i + 1] - offsets[i]), out + 2 * i);
}

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

typedef struct {
    const uint8_t *keys;
    uint32_t key_len;
    uint64_t first, count, passes;
    uint64_t fold;
} loop_arg;

/* The test.9 put/get loop shape (src/test.9.shf.c:428-431): one
 * shf_make_hash() per key, result consumed from the thread-local shf_hash.
 * The table operation is not run: the reference table engine does not travel
 * to the GPU box and this is the hash stage alone. */
static void *loop_run(void *p)
{
    loop_arg *a = (loop_arg *)p;
    uint64_t fold = 0;
    for (uint64_t pass = 0; pass < a->passes; ++pass) {
        const uint8_t *k = a->keys + a->first * a->key_len;
        for (uint64_t i = 0; i < a->count; ++i, k += a->key_len) {
            shf_make_hash((const char *)k, a->key_len);
            fold += shf_hash.u64[0] ^ shf_hash.u64[1];
        }
    }
    a->fold = fold;
    return NULL;
}

/* Returns wall seconds for `passes` passes over n keys on `threads` threads
 * (even key ranges); *fold receives a checksum so the work is observable. */
double ref_bench_make_hash_loop(const uint8_t *keys, uint32_t key_len, uint64_t n, uint64_t passes,
                                int threads, uint64_t *fold)
{
    if (threads < 1) threads = 1;
    pthread_t *tid = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    loop_arg *args = (loop_arg *)calloc((size_t)threads, sizeof(loop_arg));
    double t0 = now_s();
    for (int t = 0; t < threads; ++t) {
        uint64_t lo = n * (uint64_t)t / (uint64_t)threads, hi = n * (uint64_t)(t + 1) / (uint64_t)threads;
        args[t] = (loop_arg){keys, key_len, lo, hi - lo, passes, 0};
        pthread_create(&tid[t], NULL, loop_run, &args[t]);
    }
    uint64_t f = 0;
    for (int t = 0; t < threads; ++t) {
        pthread_join(tid[t], NULL);
        f += args[t].fold;
    }
    double dt = now_s() - t0;
    if (fold) *fold = f;
    free(tid);
    free(args);
    return dt;
}

/* ---- drop-in check: GPU hashes through the reference's caller-supplied-hash
 * seam (src/test.9.shf.c:176-182), read back through its own shf_make_hash().
 *
 * Reference API used (src/shf.h:373-437; SHF is opaque here):
 *   shf_init, shf_attach, shf_set_is_lockable, shf_put_key_val,
 *   shf_get_key_val_copy, shf_del; thread-locals shf_hash_key(_len),
 *   shf_val, shf_val_len (src/shf.private.h:187-189, src/shf.h:363-364). */
typedef struct SHF SHF;
extern void shf_init(void);
extern SHF *shf_attach(const char *path, const char *name, uint32_t delete_upon_process_exit);
extern void shf_set_is_lockable(SHF *shf, uint32_t is_lockable);
extern uint32_t shf_put_key_val(SHF *shf, const char *val, uint32_t val_len);
extern uint32_t shf_get_key_val_copy(SHF *shf);
extern uint32_t shf_del_key_val(SHF *shf);
extern char *shf_del(SHF *shf);
extern __thread const char *shf_hash_key;
extern __thread uint32_t shf_hash_key_len;
extern __thread char *shf_val;
extern __thread uint32_t shf_val_len;

#define REF_RET_KEY_FOUND 1u /* SHF_RET_KEY_FOUND, src/shf.h:345 */
#define REF_RET_KEY_PUT 8u   /* SHF_RET_KEY_PUT,   src/shf.h:348 */

/* The helper a maintainer adds next to shf_make_hash():
 * install a precomputed SHF_HASH for `key` in the thread-local seam. */
static void ref_use_hash(const char *key, uint32_t key_len, const uint64_t h[2])
{
    shf_hash.u64[0] = h[0];
    shf_hash.u64[1] = h[1];
    shf_hash_key = key;
    shf_hash_key_len = key_len;
}

/* mode 0: put with the supplied hashes, get with the reference shf_make_hash();
 * mode 1: put with shf_make_hash(), get and del with the supplied hashes.
 * Returns the number of keys found with the right value (n when the supplied
 * hashes equal the reference's), or -1 if the store could not be created. */
int64_t ref_roundtrip_with_hashes(const char *folder, const char *name, const uint8_t *bytes,
                                  const uint64_t *offsets, uint64_t n, const uint64_t *hashes, int mode)
{
    shf_init();
    SHF *shf = shf_attach(folder, name, 0);
    if (!shf) return -1;
    shf_set_is_lockable(shf, 0);
    int64_t good = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const char *k = (const char *)bytes + offsets[i];
        const uint32_t kl = (uint32_t)(offsets[i + 1] - offsets[i]);
        if (mode == 0) ref_use_hash(k, kl, hashes + 2 * i);
        else shf_make_hash(k, kl);
        if (shf_put_key_val(shf, (const char *)&i, sizeof(i)) != REF_RET_KEY_PUT) break;
    }
    for (uint64_t i = 0; i < n; ++i) {
        const char *k = (const char *)bytes + offsets[i];
        const uint32_t kl = (uint32_t)(offsets[i + 1] - offsets[i]);
        if (mode == 0) shf_make_hash(k, kl);
        else ref_use_hash(k, kl, hashes + 2 * i);
        if (shf_get_key_val_copy(shf) == REF_RET_KEY_FOUND && shf_val_len == sizeof(i) &&
            memcmp(shf_val, &i, sizeof(i)) == 0)
            ++good;
        if (mode == 1) {
            ref_use_hash(k, kl, hashes + 2 * i);
            (void)shf_del_key_val(shf);
        }
    }
    (void)shf_del(shf);
    return good;
}
