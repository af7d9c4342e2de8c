/*
 * TEST INFRASTRUCTURE ONLY -- CPU oracle for SharedHashFile's key hash.
 * See murmur3_oracle.h for the scope rule (tests / smoke / bench cpu_baseline
 * only) and for how this restatement is pinned to the reference.
 *
 * This is an independent restatement, written against the published
 * MurmurHash3 x64_128 algorithm as the reference uses it; each step cites the
 * reference line it must agree with (/root/reference/src/murmurhash3.c).
 * It is deliberately plain and portable (explicit little-endian byte
 * assembly, a byte loop for the tail) rather than fast.
 */
#include "murmur3_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* murmurhash3.c:84-85 */
#define MM3_C1 0x87c37b91114253d5ULL
#define MM3_C2 0x4cf5ad432745937fULL
/* murmurhash3.c:99 and :103 (the "*5 + n" constants of the h1 / h2 chains) */
#define MM3_N1 0x52dce729ULL
#define MM3_N2 0x38495ab5ULL
/* murmurhash3.c:65 and :67 (fmix64 multipliers) */
#define MM3_F1 0xff51afd7ed558ccdULL
#define MM3_F2 0xc4ceb9fe1a85ec53ULL

static inline uint64_t rot_left(uint64_t v, unsigned s) /* murmurhash3.c:22-25 */
{
    return (v << s) | (v >> (64u - s));
}

/* getblock64 (murmurhash3.c:41-44) reads a native u64; the reference only
 * builds on little-endian x86-64, so assemble the bytes little-endian. */
static inline uint64_t read_le64(const uint8_t *p)
{
    uint64_t v = 0;
    for (int b = 7; b >= 0; --b) v = (v << 8) | p[b];
    return v;
}

/* per-lane block mixes: murmurhash3.c:97 (k1 lane) and :101 (k2 lane) */
static inline uint64_t mix_lane1(uint64_t k) { return rot_left(k * MM3_C1, 31) * MM3_C2; }
static inline uint64_t mix_lane2(uint64_t k) { return rot_left(k * MM3_C2, 33) * MM3_C1; }

static inline uint64_t avalanche(uint64_t k) /* fmix64, murmurhash3.c:62-71 */
{
    k = (k ^ (k >> 33)) * MM3_F1;
    k = (k ^ (k >> 33)) * MM3_F2;
    return k ^ (k >> 33);
}

void oracle_murmur3_x64_128(const void *key, int len, uint32_t seed, uint64_t out[2])
{
    const uint8_t *bytes = (const uint8_t *)key;
    const int full = len / 16;                 /* murmurhash3.c:79 */
    uint64_t a = seed, b = seed;               /* h1, h2: murmurhash3.c:81-82 */

    for (int blk = 0; blk < full; ++blk) {     /* body: murmurhash3.c:92-104 */
        const uint8_t *p = bytes + 16 * blk;
        a ^= mix_lane1(read_le64(p));
        a = (rot_left(a, 27) + b) * 5 + MM3_N1;
        b ^= mix_lane2(read_le64(p + 8));
        b = (rot_left(b, 31) + a) * 5 + MM3_N2;
    }

    /* tail: murmurhash3.c:109-138. Bytes 8..14 go into the k2 lane and bytes
     * 0..7 into the k1 lane, little-endian, unsigned (no sign extension). */
    const int rem = len & 15;
    const uint8_t *t = bytes + 16 * full;
    uint64_t t1 = 0, t2 = 0;
    for (int i = rem - 1; i >= 8; --i) t2 = (t2 << 8) | t[i];
    for (int i = (rem < 8 ? rem : 8) - 1; i >= 0; --i) t1 = (t1 << 8) | t[i];
    if (rem > 8) b ^= mix_lane2(t2);
    if (rem > 0) a ^= mix_lane1(t1);

    /* finalization: murmurhash3.c:147-156. `h ^= len` promotes the int len
     * to uint64 (sign-extended for int, which only matters for len < 0). */
    const uint64_t l64 = (uint64_t)(int64_t)len;
    a ^= l64;
    b ^= l64;
    a += b;
    b += a;
    a = avalanche(a);
    b = avalanche(b);
    a += b;
    b += a;
    out[0] = a;                                /* murmurhash3.c:158-159 */
    out[1] = b;
}

void oracle_hash_fixed(const void *keys, uint32_t key_len, uint64_t n, uint32_t seed, void *out)
{
    const uint8_t *k = (const uint8_t *)keys;
    uint64_t *o = (uint64_t *)out;
    for (uint64_t i = 0; i < n; ++i)
        oracle_murmur3_x64_128(k + i * (uint64_t)key_len, (int)key_len, seed, o + 2 * i);
}

void oracle_hash_var(const void *bytes, const uint64_t *offsets, uint64_t n, uint32_t seed, void *out)
{
    const uint8_t *k = (const uint8_t *)bytes;
    uint64_t *o = (uint64_t *)out;
    for (uint64_t i = 0; i < n; ++i)
        oracle_murmur3_x64_128(k + offsets[i], (int)(offsets[i + 1] - offsets[i]), seed, o + 2 * i);
}

typedef struct {
    const uint8_t *keys;
    uint32_t key_len;
    uint64_t first, count;
    uint32_t seed;
    uint64_t *out;
} fixed_range;

static void *fixed_range_run(void *arg)
{
    fixed_range *r = (fixed_range *)arg;
    oracle_hash_fixed(r->keys + r->first * r->key_len, r->key_len, r->count, r->seed, r->out + 2 * r->first);
    return NULL;
}

void oracle_hash_fixed_mt(const void *keys, uint32_t key_len, uint64_t n, uint32_t seed, void *out, int threads)
{
    if (threads < 1) threads = 1;
    pthread_t *tid = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    fixed_range *rng = (fixed_range *)calloc((size_t)threads, sizeof(fixed_range));
    for (int t = 0; t < threads; ++t) {
        uint64_t lo = n * (uint64_t)t / (uint64_t)threads, hi = n * (uint64_t)(t + 1) / (uint64_t)threads;
        rng[t] = (fixed_range){(const uint8_t *)keys, key_len, lo, hi - lo, seed, (uint64_t *)out};
        pthread_create(&tid[t], NULL, fixed_range_run, &rng[t]);
    }
    for (int t = 0; t < threads; ++t) pthread_join(tid[t], NULL);
    free(tid);
    free(rng);
}

/* shf.c:800-803 (put) and :893-896 (find):
 *   win  = u16[0] % 256, tab2 = u16[1] % 2048, row = u16[2] % 512,
 *   rnd  = u32[2] % 2^21
 * packed as SHF_UID's bit layout (shf.private.h:170-178: win 8 | tab 11 |
 * row 9 | ref 4, ref left 0) in the low word and rnd in the high word. */
uint64_t oracle_uid_parts(const uint64_t h[2])
{
    const uint64_t win = (h[0] >> 0) & 0xffff;
    const uint64_t tab = (h[0] >> 16) & 0xffff;
    const uint64_t row = (h[0] >> 32) & 0xffff;
    const uint64_t rnd = h[1] & 0xffffffffULL;
    return (win % 256) | ((tab % 2048) << 8) | ((row % 512) << 19) | ((rnd % (1u << 21)) << 32);
}

void oracle_uid_parts_batch(const void *hashes, uint64_t n, uint64_t *parts)
{
    const uint64_t *h = (const uint64_t *)hashes;
    for (uint64_t i = 0; i < n; ++i) parts[i] = oracle_uid_parts(h + 2 * i);
}

/* shf_find_key_internal(), SHF_UID_NONE branch (shf.c:886-922), up to the key
 * compare:
 *   win  = shf_hash.u16[0] % 256        shf.c:893
 *   tab2 = shf_hash.u16[1] % 2048       shf.c:894
 *   row  = shf_hash.u16[2] % 512        shf.c:895
 *   rnd  = shf_hash.u32[2] % 2^21       shf.c:896
 *   tab  = wins[win].tabs[tab2].tab     shf.c:906 (the index folds it into tab_slot)
 *   for ref in 0..15: candidate if pos != 0 && ref.rnd == rnd && ref.tab == tab2  shf.c:918-921
 * SHF_REF_MMAP (shf.private.h:48-52): a packed u32 bitfield tab:11 then rnd:21
 * (gcc allocates from bit 0 on x86-64), then u32 pos. The uid of a hit is
 * SHF_UID with ref = the first candidate (shf.c:931-932, shf.private.h:170-178). */
void oracle_probe(const void *hashes, uint64_t n, const uint32_t *tab_slot, const void *rows, uint64_t n_slots,
                  uint32_t *out)
{
    const uint64_t *h = (const uint64_t *)hashes;
    const uint8_t *rb = (const uint8_t *)rows;
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t h1 = h[2 * i], h2 = h[2 * i + 1];
        const uint32_t win = (uint32_t)((h1 & 0xffff) % 256);
        const uint32_t tab2 = (uint32_t)(((h1 >> 16) & 0xffff) % 2048);
        const uint32_t row = (uint32_t)(((h1 >> 32) & 0xffff) % 512);
        const uint32_t rnd = (uint32_t)((h2 & 0xffffffffu) % (1u << 21));
        uint32_t *o = out + 4 * i;
        o[0] = 0xffffffffu;
        o[1] = 0;
        o[2] = 0xffffu << 16;
        o[3] = 0xffffffffu;
        const uint32_t e = tab_slot[(win << 11) | tab2];
        if (e == 0xffffffffu || (uint64_t)(e >> 11) >= n_slots) continue;
        const uint32_t slot = e >> 11, tab = e & 0x7ff;
        const uint8_t *r = rb + (uint64_t)slot * 65536u + (uint64_t)row * 128u;
        uint32_t mask = 0, first = 16, pos = 0;
        for (uint32_t ref = 0; ref < 16; ++ref) {
            uint32_t word, rpos;
            memcpy(&word, r + 8 * ref, 4);
            memcpy(&rpos, r + 8 * ref + 4, 4);
            const uint32_t ref_tab = word & 0x7ff, ref_rnd = word >> 11;
            if (rpos != 0 && ref_rnd == rnd && ref_tab == tab2) {
                mask |= 1u << ref;
                if (first == 16) {
                    first = ref;
                    pos = rpos;
                }
            }
        }
        if (mask) o[0] = win | (tab2 << 8) | (row << 19) | (first << 28);
        o[1] = pos;
        o[2] = mask | (tab << 16);
        o[3] = slot;
    }
}

/* SMHasher VerificationTest: hash keys {0}, {0,1}, ... of length i with seed
 * 256 - i, then hash the 256 concatenated 16-byte results with seed 0 and
 * read the first 4 bytes little-endian. */
uint32_t oracle_smhasher_verification(void)
{
    uint8_t key[256];
    uint8_t all[256 * 16];
    for (int i = 0; i < 256; ++i) {
        uint64_t h[2];
        key[i] = (uint8_t)i;
        oracle_murmur3_x64_128(key, i, 256u - (uint32_t)i, h);
        for (int b = 0; b < 8; ++b) {
            all[16 * i + b] = (uint8_t)(h[0] >> (8 * b));
            all[16 * i + 8 + b] = (uint8_t)(h[1] >> (8 * b));
        }
    }
    uint64_t fin[2];
    oracle_murmur3_x64_128(all, 256 * 16, 0, fin);
    return (uint32_t)(fin[0] & 0xffffffffu);
}
