/*
 * The drop-in seam for C++ callers, proven from a g++-compiled program (no
 * ctypes): libshf_hash_batch.so (the product) linked with the reference's own
 * SharedHashFile class (src/SharedHashFile.cpp) and table engine (src/shf.c +
 * src/murmurhash3.c), all compiled by oracle/Makefile into oracle/_ref/.
 *
 *   1. test.a.shf.cpp:172-270's caller-supplied-hash block, with the hashes
 *      coming from one GPU batch (shf_hash_batch::HashVar) instead of hand
 *      values: for keys "foo", "bar" and two 32-byte binary keys, the GPU
 *      record equals what SharedHashFile::MakeHash leaves in shf_hash, then
 *      UseHash + PutKeyVal / GetUidValCopy / GetKeyValCopy / GetKeyKeyCopy /
 *      GetUidKeyCopy / DelKeyVal behave as with MakeHash;
 *   2. shf_hash_batch::PutBatch of n variable-length keys through the class,
 *      then the reference's own MakeHash + GetKeyValCopy finds every one with
 *      its value (and none of n/10 absent keys);
 *   3. fixed 16-byte keys: HashFixed + UseHash + PutKeyVal, found again by
 *      MakeHash + GetKeyValCopy.
 *
 * TEST INFRASTRUCTURE: built by tests/c/Makefile where /root/reference exists
 * (the reference's headers are needed to compile it), into tests/c/build/,
 * which travels to the GPU box with the tree. Exit status: 0 pass, 1 fail,
 * 2 no usable GPU (the library refused: no CPU fallback).
 */
#include <ftw.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <string>
#include <vector>

#include "SharedHashFile.hpp"
#include "shf_hash_batch_shf.hpp"

namespace {

uint64_t splitmix(uint64_t &s)
{
    uint64_t z = (s += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

int failures = 0;
int checks = 0;

void expect(bool ok, const std::string &what)
{
    ++checks;
    if (!ok) {
        ++failures;
        fprintf(stderr, "test_seam_cpp: FAIL: %s\n", what.c_str());
    }
}

int remove_entry(const char *path, const struct stat *, int, struct FTW *) { return remove(path); }

}  // namespace

int main(int argc, char **argv)
{
    const uint64_t n_put = argc > 1 ? strtoull(argv[1], 0, 10) : 100000, n_absent = n_put / 10;
    const int rc0 = shf_hash_batch_check_device();
    if (rc0 != SHF_HB_OK) {
        fprintf(stderr, "test_seam_cpp: no usable GPU: %s\n", shf_hash_batch_strerror(rc0));
        return 2;
    }
    char folder[] = "/dev/shm/seamcppXXXXXX";
    if (!mkdtemp(folder)) {
        perror("mkdtemp");
        return 1;
    }
    SharedHashFile shf;
    expect(shf.Attach(folder, "seamcpp", 0), "Attach");

    /* 1. the own-hash block, hashes from one GPU batch */
    std::string key32a(32, '\0'), key32b(32, '\0');
    uint64_t st = 0x5348460000000091ull;
    for (int b = 0; b < 32; b += 8) {
        const uint64_t x = splitmix(st), y = splitmix(st);
        memcpy(&key32a[b], &x, 8);
        memcpy(&key32b[b], &y, 8);
    }
    const std::vector<std::string> keys = {"foo", "bar", key32a, key32b};
    std::string packed;
    std::vector<uint64_t> off = {0};
    for (const auto &k : keys) {
        packed += k;
        off.push_back(packed.size());
    }
    std::vector<shf_hash128> h;
    expect(shf_hash_batch::HashVar(packed.data(), off.data(), keys.size(), h) == SHF_HB_OK, "HashVar (own-hash keys)");
    for (size_t i = 0; i < keys.size() && !failures; ++i) {
        const char *k = packed.data() + off[i];
        const uint32_t kl = (uint32_t)keys[i].size();
        const std::string tag = "key " + std::to_string(i) + ": ";
        shf.MakeHash(k, kl);
        expect(shf_hash.u64[0] == h[i].h1 && shf_hash.u64[1] == h[i].h2, tag + "GPU record == MakeHash's shf_hash");
        shf_hash_batch::UseHash(k, kl, h[i]);
        expect(shf.PutKeyVal("val", 3) == SHF_RET_KEY_PUT, tag + "PutKeyVal");
        const uint32_t uid = shf_uid;
        expect(uid != SHF_UID_NONE, tag + "uid set");
        expect(shf.GetUidValCopy(uid) == SHF_RET_KEY_FOUND && shf_val_len == 3 && memcmp(shf_val, "val", 3) == 0,
               tag + "GetUidValCopy");
        shf_hash_batch::UseHash(k, kl, h[i]);
        expect(shf.GetKeyValCopy() == SHF_RET_KEY_FOUND && shf_val_len == 3 && memcmp(shf_val, "val", 3) == 0 &&
                   shf_uid == uid,
               tag + "GetKeyValCopy");
        expect(shf.GetKeyKeyCopy() == SHF_RET_KEY_FOUND && shf_key_len == kl && memcmp(shf_key, k, kl) == 0,
               tag + "GetKeyKeyCopy");
        expect(shf.GetUidKeyCopy(uid) == SHF_RET_KEY_FOUND && shf_key_len == kl && memcmp(shf_key, k, kl) == 0,
               tag + "GetUidKeyCopy");
        shf_hash_batch::UseHash(k, kl, h[i]);
        expect(shf.DelKeyVal() == SHF_RET_KEY_FOUND, tag + "DelKeyVal");
        shf_hash_batch::UseHash(k, kl, h[i]);
        expect(shf.GetKeyValCopy() == SHF_RET_KEY_NONE, tag + "gone after DelKeyVal");
    }

    /* 2. PutBatch through the class, the reference's own MakeHash get finds them */
    const uint64_t n = n_put + n_absent;
    std::vector<uint64_t> koff(n + 1, 0), voff(n + 1, 0);
    for (uint64_t i = 0; i < n; ++i) {
        koff[i + 1] = koff[i] + 4 + splitmix(st) % 64;
        voff[i + 1] = voff[i] + 8;
    }
    std::vector<char> bytes(koff[n] + 8), vals(8 * n);
    for (uint64_t b = 0; b < koff[n]; b += 8) {
        const uint64_t v = splitmix(st);
        memcpy(&bytes[b], &v, 8);
    }
    for (uint64_t i = 0; i < n; ++i) {  /* unique keys: the index in their first 4-8 bytes */
        const uint64_t len = koff[i + 1] - koff[i];
        memcpy(&bytes[koff[i]], &i, len < 8 ? len : 8);
        memcpy(&vals[8 * i], &i, 8);
    }
    const int64_t put = shf_hash_batch::PutBatch(shf, bytes.data(), koff.data(), n_put, vals.data(), voff.data());
    expect(put == (int64_t)n_put, "PutBatch put every key");
    uint64_t found = 0, right = 0, absent_found = 0;
    for (uint64_t i = 0; i < n; ++i) {
        shf.MakeHash(&bytes[koff[i]], (uint32_t)(koff[i + 1] - koff[i]));
        if (shf.GetKeyValCopy() != SHF_RET_KEY_FOUND) continue;
        uint64_t v = 0;
        memcpy(&v, shf_val, 8);
        if (i < n_put) {
            ++found;
            right += shf_val_len == 8 && v == i;
        } else {
            ++absent_found;
        }
    }
    expect(found == n_put && right == n_put && absent_found == 0, "MakeHash get after PutBatch");

    /* 3. fixed 16-byte keys */
    const uint64_t nf = n_put / 2;
    std::vector<uint8_t> fk(16 * nf);
    for (uint64_t i = 0; i < nf; ++i) {
        const uint64_t a = splitmix(st) | 1ull << 63, b = i;  /* high bit: never a key of part 2's shape */
        memcpy(&fk[16 * i], &a, 8);
        memcpy(&fk[16 * i + 8], &b, 8);
    }
    std::vector<shf_hash128> hf;
    expect(shf_hash_batch::HashFixed(fk.data(), 16, nf, hf) == SHF_HB_OK, "HashFixed");
    uint64_t fixed_put = 0, fixed_found = 0;
    for (uint64_t i = 0; i < nf; ++i) {
        shf_hash_batch::UseHash(reinterpret_cast<const char *>(&fk[16 * i]), 16, hf[i]);
        fixed_put += shf.PutKeyVal(reinterpret_cast<const char *>(&i), 8) == SHF_RET_KEY_PUT;
    }
    for (uint64_t i = 0; i < nf; ++i) {
        shf.MakeHash(reinterpret_cast<const char *>(&fk[16 * i]), 16);
        uint64_t v = ~0ull;
        if (shf.GetKeyValCopy() == SHF_RET_KEY_FOUND && shf_val_len == 8) memcpy(&v, shf_val, 8);
        fixed_found += v == i;
    }
    expect(fixed_put == nf && fixed_found == nf, "fixed 16-B keys: UseHash put, MakeHash get");

    /* 4. the same keys' 8-B UID parts (shf_uid_parts_batch_fixed) through UseUidParts: GetKeyValCopy finds each */
    std::vector<uint64_t> parts(nf);
    uint64_t parts_found = 0;
    if (shf_uid_parts_batch_fixed(fk.data(), 16, nf, SHF_HASH_BATCH_SEED, parts.data(), SHF_HASH_MEM_HOST) ==
        SHF_HB_OK) {
        for (uint64_t i = 0; i < nf; ++i) {
            shf_hash_batch::UseUidParts(reinterpret_cast<const char *>(&fk[16 * i]), 16, parts[i]);
            uint64_t v = ~0ull;
            if (shf.GetKeyValCopy() == SHF_RET_KEY_FOUND && shf_val_len == 8) memcpy(&v, shf_val, 8);
            parts_found += v == i;
        }
    }
    expect(parts_found == nf, "fixed 16-B keys: UID parts through UseUidParts, GetKeyValCopy");

    /* the store's files go with the folder (shf_del would run `du` and `rm` through popen) */
    shf.Detach();
    nftw(folder, remove_entry, 16, FTW_DEPTH | FTW_PHYS);
    printf("{\"checks\": %d, \"failures\": %d, \"own_hash_keys\": %zu, \"n_put\": %llu, \"found\": %llu, "
           "\"right\": %llu, \"absent_found\": %llu, \"fixed_found\": %llu, \"parts_found\": %llu}\n",
           checks, failures, keys.size(), (unsigned long long)n_put, (unsigned long long)found,
           (unsigned long long)right, (unsigned long long)absent_found, (unsigned long long)fixed_found,
           (unsigned long long)parts_found);
    return failures ? 1 : 0;
}
