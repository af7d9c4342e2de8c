#!/usr/bin/env python3
"""Generate the golden vectors for the batch key-hashing path.

Run HERE (the build container), where /root/reference exists:

    make -C oracle ref && python tests/golden/make_golden.py

Every expected hash below is produced by the REFERENCE's own code,
oracle/_ref/libref_shf.so = /root/reference/src/murmurhash3.c + shf.c built by
oracle/Makefile, read through:
  * ref_make_hash_into(key, len, out): calls the reference shf_make_hash()
    (src/shf.c:450-462, seed 12345) and copies the thread-local shf_hash
    (src/shf.private.h:180-189);
  * ref_murmur3_into(key, len, seed, out): MurmurHash3_x64_128
    (src/murmurhash3.c:75-160) for seeds other than 12345.

Outputs (data only: inputs and expected outputs):
  tests/golden/murmur3_golden.json   small cases, key bytes inline as hex
  tests/golden/murmur3_var.npz       1,024 variable-length keys (bytes,
                                     offsets, hashes) for the var-len path
"""
import ctypes
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from sharedhashfile_amd.keygen import splitmix_bytes, splitmix_lengths  # noqa: E402

SEED = 12345  # src/shf.c:456


def load_ref():
    path = os.path.join(ROOT, "oracle", "_ref", "libref_shf.so")
    lib = ctypes.CDLL(path)
    lib.ref_make_hash_into.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64)]
    lib.ref_murmur3_into.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64)]
    lib.ref_hash_var.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
    return lib


def ref_make_hash(lib, key: bytes):
    out = (ctypes.c_uint64 * 2)()
    lib.ref_make_hash_into(key, len(key), out)
    return int(out[0]), int(out[1])


def ref_murmur(lib, key: bytes, seed: int):
    out = (ctypes.c_uint64 * 2)()
    lib.ref_murmur3_into(key, len(key), seed, out)
    return int(out[0]), int(out[1])


def hx(v):
    return "%016x" % v


def uid_parts(h1, h2):
    """shf.c:800-803 hash-bit consumers, packed as include/shf_hash_batch.h."""
    win = (h1 & 0xFFFF) % 256
    tab = ((h1 >> 16) & 0xFFFF) % 2048
    row = ((h1 >> 32) & 0xFFFF) % 512
    rnd = (h2 & 0xFFFFFFFF) % (1 << 21)
    return win | (tab << 8) | (row << 19) | (rnd << 32)


def main():
    lib = load_ref()
    cases = []

    # 1. key bytes 0,1,2,... at every len&15 class (SURVEY.md s8(a) golden sample).
    lens = list(range(0, 65)) + [127, 128, 129, 255, 256, 257, 511, 512, 1000, 4096, 65537]
    for n in lens:
        key = bytes(i & 0xFF for i in range(n))
        h1, h2 = ref_make_hash(lib, key)
        cases.append({"name": "seq_%d" % n, "seed": SEED, "key_hex": key.hex(), "h1": hx(h1), "h2": hx(h2)})

    # 2. the README example key and the SHA-256 test keys of src/test.9.shf.c:175-232.
    for key in [b"key", b"foo", b"bar", b"", b"a" * 31]:
        h1, h2 = ref_make_hash(lib, key)
        cases.append({"name": "str_%s" % key[:8].decode(), "seed": SEED, "key_hex": key.hex(),
                      "h1": hx(h1), "h2": hx(h2), "uid_parts": "%016x" % uid_parts(h1, h2)})

    # 3. other seeds (the batch ABI exposes the seed; shf_make_hash fixes 12345).
    for seed in [0, 1, 0x7FFFFFFF, 0x80000000, 0xFFFFFFFF]:
        for n in [0, 7, 16, 31, 256]:
            key = splitmix_bytes(n, 0x5348460000000100 + n)
            h1, h2 = ref_murmur(lib, key, seed)
            cases.append({"name": "seed_%x_%d" % (seed, n), "seed": seed, "key_hex": key.hex(),
                          "h1": hx(h1), "h2": hx(h2)})

    # 4. test.9 counter keys: the 4 LE bytes of uint32 i (src/test.9.shf.c:429),
    #    and the same counters zero-padded to 16 bytes. First 64 hashes inline,
    #    the rest as a digest of the concatenated 16-byte SHF_HASH records.
    counters = {}
    for width, count in [(4, 100000), (16, 100000)]:
        keys = np.zeros((count, width), dtype=np.uint8)
        keys[:, :4] = np.arange(count, dtype="<u4").view(np.uint8).reshape(count, 4)
        off = np.arange(count + 1, dtype=np.uint64) * width
        out = np.zeros((count, 2), dtype=np.uint64)
        flat = np.ascontiguousarray(keys.reshape(-1))
        lib.ref_hash_var(flat.ctypes.data, off.ctypes.data, count, out.ctypes.data)
        counters["counter_w%d" % width] = {
            "key_len": width, "count": count, "seed": SEED,
            "first_h1": [hx(int(v)) for v in out[:64, 0]],
            "first_h2": [hx(int(v)) for v in out[:64, 1]],
            "sha256_of_hashes": hashlib.sha256(out.astype("<u8").tobytes()).hexdigest(),
        }

    # 5. fixed 16 B and 256 B random keys (the bench configs' key shapes).
    fixed = {}
    for width, count, stream in [(16, 4096, 0x5348460000000001), (256, 1024, 0x5348460000000002)]:
        flat = np.frombuffer(splitmix_bytes(width * count, stream), dtype=np.uint8).copy()
        off = np.arange(count + 1, dtype=np.uint64) * width
        out = np.zeros((count, 2), dtype=np.uint64)
        lib.ref_hash_var(flat.ctypes.data, off.ctypes.data, count, out.ctypes.data)
        fixed["fixed_w%d" % width] = {
            "key_len": width, "count": count, "splitmix_stream": "%x" % stream, "seed": SEED,
            "sha256_of_keys": hashlib.sha256(flat.tobytes()).hexdigest(),
            "sha256_of_hashes": hashlib.sha256(out.astype("<u8").tobytes()).hexdigest(),
            "first_h1": [hx(int(v)) for v in out[:16, 0]],
            "first_h2": [hx(int(v)) for v in out[:16, 1]],
        }

    doc = {
        "generator": "tests/golden/make_golden.py",
        "reference": "oracle/_ref/libref_shf.so built from /root/reference/src/{murmurhash3.c,shf.c}",
        "smhasher_verification": "6384ba69",
        "cases": cases,
        "counters": counters,
        "fixed": fixed,
    }
    with open(os.path.join(HERE, "murmur3_golden.json"), "w") as f:
        json.dump(doc, f, indent=1)

    # 6. variable-length keys 0..600 B, packed, every len&15 class present.
    n = 1024
    lens = splitmix_lengths(n, 0, 600, 0x5348460000000003)
    lens[:16] = np.arange(16) + 16 * 3  # force every len&15 class
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens.astype(np.uint64))
    flat = np.frombuffer(splitmix_bytes(int(off[-1]), 0x5348460000000004), dtype=np.uint8).copy()
    out = np.zeros((n, 2), dtype=np.uint64)
    lib.ref_hash_var(flat.ctypes.data, off.ctypes.data, n, out.ctypes.data)
    np.savez_compressed(os.path.join(HERE, "murmur3_var.npz"), bytes=flat, offsets=off, hashes=out)
    print("wrote", len(cases), "cases;", n, "var keys;", int(off[-1]), "bytes")


if __name__ == "__main__":
    main()
