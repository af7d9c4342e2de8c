/* TEST INFRASTRUCTURE: the C oracle (oracle/murmur3_oracle.c) under
 * -fsanitize=address,undefined (tests/c/Makefile target `sanitize`), run by
 * tests/test_host_plan.py on the CPU.
 *
 * stdin: one golden case per line, "seed key_hex h1_hex h2_hex" (key_hex "-"
 * for the empty key), from tests/golden/murmur3_golden.json (the reference's
 * own hashes). Each key is hashed from a heap buffer of exactly its length, so
 * an over-read of the tail (murmurhash3.c:109-138) is an ASan report; then the
 * same keys go through the batch entry points (packed fixed-length runs and one
 * variable-length batch, both in exact-size buffers) and SMHasher's
 * verification value is recomputed. Exit 0 = all equal and no sanitizer report. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/murmur3_oracle.h"

static int hexval(int c) { return c <= '9' ? c - '0' : (c | 32) - 'a' + 10; }

int main(void) {
  char *line = NULL;
  size_t cap = 0;
  unsigned seed;
  unsigned long long h1, h2;
  int cases = 0, bad = 0;
  uint8_t *all = NULL;
  uint64_t *off = malloc(sizeof(uint64_t));
  uint64_t *want = NULL, total = 0;
  off[0] = 0;
  while (getline(&line, &cap, stdin) > 0) {
    char *save = NULL, *f0 = strtok_r(line, " \n", &save), *khex = strtok_r(NULL, " \n", &save);
    char *f2 = strtok_r(NULL, " \n", &save), *f3 = strtok_r(NULL, " \n", &save);
    if (!f0 || !khex || !f2 || !f3) continue;
    seed = (unsigned)strtoul(f0, NULL, 10);
    h1 = strtoull(f2, NULL, 16);
    h2 = strtoull(f3, NULL, 16);
    const size_t len = strcmp(khex, "-") ? strlen(khex) / 2 : 0;
    uint8_t *key = malloc(len ? len : 1);
    for (size_t i = 0; i < len; ++i) key[i] = (uint8_t)(hexval(khex[2 * i]) << 4 | hexval(khex[2 * i + 1]));
    uint64_t out[2];
    oracle_murmur3_x64_128(len ? key : NULL, (int)len, seed, out);
    if (out[0] != h1 || out[1] != h2) {
      fprintf(stderr, "case %d (len %zu): %016llx %016llx != %016llx %016llx\n", cases, len,
              (unsigned long long)out[0], (unsigned long long)out[1], h1, h2);
      ++bad;
    }
    if (seed == 12345u) { /* the seed-12345 cases also go through the batch entry points */
      all = realloc(all, total + len + 1);
      if (len) memcpy(all + total, key, len);
      total += len;
      const int k = (int)(want ? want[0] : 0);
      want = realloc(want, (size_t)(2 * (k + 1) + 1) * sizeof(uint64_t));
      if (!k) want[0] = 0;
      want[1 + 2 * k] = h1;
      want[2 + 2 * k] = h2;
      want[0] = k + 1;
      off = realloc(off, (size_t)(k + 2) * sizeof(uint64_t));
      off[k + 1] = total;
      /* the key alone as a fixed-length batch of one, exact-size output */
      uint64_t *o1 = malloc(16);
      oracle_hash_fixed(key, (uint32_t)len, 1, 12345u, o1);
      if (o1[0] != h1 || o1[1] != h2) ++bad;
      free(o1);
    }
    free(key);
    ++cases;
  }
  const uint64_t n = want ? want[0] : 0;
  if (n) {
    uint8_t *exact = malloc(total ? total : 1); /* exact size: the last key's tail ends the buffer */
    memcpy(exact, all, total);
    uint64_t *out = malloc((size_t)n * 16);
    oracle_hash_var(exact, off, n, 12345u, out);
    for (uint64_t i = 0; i < n; ++i)
      if (out[2 * i] != want[1 + 2 * i] || out[2 * i + 1] != want[2 + 2 * i]) ++bad;
    uint64_t *parts = malloc((size_t)n * 8);
    oracle_uid_parts_batch(out, n, parts);
    for (uint64_t i = 0; i < n; ++i)
      if (parts[i] != oracle_uid_parts(out + 2 * i)) ++bad;
    free(parts);
    free(out);
    free(exact);
  }
  const uint32_t v = oracle_smhasher_verification();
  if (v != 0x6384BA69u) {
    fprintf(stderr, "smhasher verification %08x\n", v);
    ++bad;
  }
  free(line);
  free(all);
  free(off);
  free(want);
  printf("oracle under ASan/UBSan: %d cases, %llu in the batch, %d mismatches\n", cases, (unsigned long long)n, bad);
  return bad || cases == 0;
}
