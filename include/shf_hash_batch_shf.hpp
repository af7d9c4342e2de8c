/*
 * shf_hash_batch_shf.hpp -- the GPU batch hashes (shf_hash_batch.h) for C++
 * callers of SharedHashFile's class interface.
 *
 * The reference exposes hashing to C++ through
 *
 *     void SharedHashFile::MakeHash(const char *key, uint32_t key_len);
 *                                     -- /root/reference/src/SharedHashFile.hpp:40,
 *                                        /root/reference/src/SharedHashFile.cpp:84-91
 *
 * which is shf_make_hash() (shf.c:450-462): it fills the thread-local SHF_HASH
 * shf_hash, shf_hash_key and shf_hash_key_len that every later
 * PutKeyVal / GetKeyValCopy / GetKeyKeyCopy / DelKeyVal / AddKeyVal reads.
 * test.a.shf.cpp:172-270 sets those thread-locals by hand instead ("use own
 * hash ... instead of shf->MakeHash"); this header packages that seam for
 * batches hashed on the GPU:
 *
 *   shf_hash_batch::UseHash()    MakeHash(key, key_len) with the hash already
 *                                computed (one shf_hash128 record)
 *   shf_hash_batch::UseUidParts()  the same from an 8-B UID-parts word
 *                                (shf_uid_parts_batch_*): the SHF_HASH fields
 *                                shf.c reads, every other byte 0
 *   shf_hash_batch::HashVar()    a host batch of variable-length keys hashed on
 *   shf_hash_batch::HashFixed()  the GPU into a std::vector of records
 *   shf_hash_batch::PutBatch()   HashVar + UseHash + SharedHashFile::PutKeyVal
 *                                per key
 *
 * Like MakeHash, UseHash works on the calling thread's state, not on the
 * object (SharedHashFile.cpp:85's own note). Include it after the reference's
 * SharedHashFile.hpp (which brings in shf.private.h and shf.h). Header-only:
 * the application links libshf_hash_batch.so and nothing else.
 */
#ifndef SHF_HASH_BATCH_SHF_HPP
#define SHF_HASH_BATCH_SHF_HPP

#ifndef __SHAREDHASHFILE_HPP__
#error "include the reference's SharedHashFile.hpp before shf_hash_batch_shf.hpp"
#endif

#include <stdint.h>

#include <vector>

#include "shf_hash_batch.h"

namespace shf_hash_batch {

/* SharedHashFile::MakeHash(key, key_len) with h = that key's record from a
 * shf_hash_batch_* call (seed SHF_HASH_BATCH_SEED). The key pointer is kept,
 * not copied, as MakeHash keeps it (shf.c:460-461): it must stay valid until
 * the class call that follows. */
inline void UseHash(const char *key, uint32_t key_len, const shf_hash128 &h)
{
    shf_hash.u64[0] = h.h1;
    shf_hash.u64[1] = h.h2;
    shf_hash_key = key;
    shf_hash_key_len = key_len;
}

/* MakeHash(key, key_len) from a UID-parts word: win, tab2, row and rnd in the
 * SHF_HASH fields put/find read (/root/reference/src/shf.c:800-803, :893-896),
 * zeros elsewhere; the class calls that follow behave as with the full hash. */
inline void UseUidParts(const char *key, uint32_t key_len, uint64_t parts)
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

/* n host keys, key i = bytes[offsets[i] .. offsets[i+1]), hashed on the GPU
 * into out (resized to n). Returns SHF_HB_OK or a negative SHF_HB_ERR_*. */
inline int HashVar(const char *bytes, const uint64_t *offsets, uint64_t n, std::vector<shf_hash128> &out)
{
    out.resize(n);
    if (n == 0) return SHF_HB_OK;
    return shf_hash_batch_var(bytes, offsets, n, SHF_HASH_BATCH_SEED, out.data(), SHF_HASH_MEM_HOST);
}

/* n host keys of key_len bytes each, back to back. */
inline int HashFixed(const void *keys, uint32_t key_len, uint64_t n, std::vector<shf_hash128> &out)
{
    out.resize(n);
    if (n == 0) return SHF_HB_OK;
    return shf_hash_batch_fixed(keys, key_len, n, SHF_HASH_BATCH_SEED, out.data(), SHF_HASH_MEM_HOST);
}

/* Put n host keys with values (value i = vals[val_offsets[i] ..
 * val_offsets[i+1])): one GPU batch hash, then UseHash + shf.PutKeyVal per
 * key. Returns the keys put (n, or the index of the first PutKeyVal that did
 * not return SHF_RET_KEY_PUT), or a negative SHF_HB_ERR_* with nothing put. */
inline int64_t PutBatch(SharedHashFile &shf, const char *bytes, const uint64_t *offsets, uint64_t n,
                        const char *vals, const uint64_t *val_offsets)
{
    std::vector<shf_hash128> h;
    const int rc = HashVar(bytes, offsets, n, h);
    if (rc != SHF_HB_OK) return rc;
    uint64_t i = 0;
    for (; i < n; ++i) {
        UseHash(bytes + offsets[i], (uint32_t)(offsets[i + 1] - offsets[i]), h[i]);
        if (shf.PutKeyVal(vals + val_offsets[i], (uint32_t)(val_offsets[i + 1] - val_offsets[i])) != SHF_RET_KEY_PUT)
            break;
    }
    return (int64_t)i;
}

}  // namespace shf_hash_batch

#endif /* SHF_HASH_BATCH_SHF_HPP */
