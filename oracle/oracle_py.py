"""ctypes binding of the CPU oracle (oracle/_build/liboracle.so).

TEST INFRASTRUCTURE ONLY: used by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg as the checker; never by the product path.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "_build", "liboracle.so")
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libref_shf.so")


def _ensure_built():
    if not os.path.exists(ORACLE_SO):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "oracle"])


class Oracle:
    def __init__(self):
        _ensure_built()
        lib = ctypes.CDLL(ORACLE_SO)
        vp, u32, u64, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
        lib.oracle_murmur3_x64_128.argtypes = [vp, i32, u32, vp]
        lib.oracle_hash_fixed.argtypes = [vp, u32, u64, u32, vp]
        lib.oracle_hash_var.argtypes = [vp, vp, u64, u32, vp]
        lib.oracle_hash_fixed_mt.argtypes = [vp, u32, u64, u32, vp, i32]
        lib.oracle_uid_parts_batch.argtypes = [vp, u64, vp]
        lib.oracle_smhasher_verification.restype = u32
        self.lib = lib

    def hash(self, key: bytes, seed=12345):
        out = (ctypes.c_uint64 * 2)()
        buf = ctypes.create_string_buffer(key, len(key))
        self.lib.oracle_murmur3_x64_128(buf, len(key), seed, out)
        return int(out[0]), int(out[1])

    def hash_fixed(self, keys, key_len=None, seed=12345, threads=1):
        keys = np.ascontiguousarray(keys).view(np.uint8)
        if key_len is None:
            n, key_len = keys.shape
        else:
            n = keys.size // key_len if key_len else 0
        out = np.empty((n, 2), dtype=np.uint64)
        if threads > 1:
            self.lib.oracle_hash_fixed_mt(keys.ctypes.data, key_len, n, seed, out.ctypes.data, threads)
        else:
            self.lib.oracle_hash_fixed(keys.ctypes.data, key_len, n, seed, out.ctypes.data)
        return out

    def hash_var(self, data, offsets, seed=12345):
        data = np.ascontiguousarray(data).view(np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        n = offsets.size - 1
        out = np.empty((n, 2), dtype=np.uint64)
        self.lib.oracle_hash_var(data.ctypes.data, offsets.ctypes.data, n, seed, out.ctypes.data)
        return out

    def uid_parts(self, hashes):
        hashes = np.ascontiguousarray(hashes, dtype=np.uint64)
        n = hashes.shape[0]
        out = np.empty((n,), dtype=np.uint64)
        self.lib.oracle_uid_parts_batch(hashes.ctypes.data, n, out.ctypes.data)
        return out

    def smhasher(self):
        return self.lib.oracle_smhasher_verification()


def reference_lib():
    """oracle/_ref/libref_shf.so (the reference's own code), or None if not built."""
    if not os.path.exists(REF_SO):
        return None
    lib = ctypes.CDLL(REF_SO)
    vp, u32, u64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64
    lib.ref_make_hash_into.argtypes = [ctypes.c_char_p, u32, vp]
    lib.ref_hash_var.argtypes = [vp, vp, u64, vp]
    lib.ref_bench_make_hash_loop.argtypes = [vp, u32, u64, u64, ctypes.c_int, ctypes.POINTER(u64)]
    lib.ref_bench_make_hash_loop.restype = ctypes.c_double
    return lib
