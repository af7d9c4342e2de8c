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
        lib.oracle_probe.argtypes = [vp, u64, vp, vp, u64, vp]
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

    def probe(self, hashes, tab_slot, rows, n_slots=None):
        """Row pre-probe records (n, 4) uint32 {uid, pos, mask | tab << 16, slot}."""
        hashes = np.ascontiguousarray(hashes, dtype=np.uint64)
        tab_slot = np.ascontiguousarray(tab_slot, dtype=np.uint32)
        rows = np.ascontiguousarray(rows).view(np.uint8).reshape(-1)
        if n_slots is None:
            n_slots = rows.size // 65536
        n = hashes.shape[0]
        out = np.empty((n, 4), dtype=np.uint32)
        self.lib.oracle_probe(hashes.ctypes.data, n, tab_slot.ctypes.data, rows.ctypes.data, n_slots, out.ctypes.data)
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
    lib.ref_probe_fixture.argtypes = [ctypes.c_char_p, ctypes.c_char_p, vp, vp, u64, u64, vp, vp, vp, u64]
    lib.ref_probe_fixture.restype = ctypes.c_int64
    lib.ref_export_rows.argtypes = [vp, vp, vp, u64]
    lib.ref_export_rows.restype = ctypes.c_int64
    lib.ref_store_open.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    lib.ref_store_open.restype = vp
    lib.ref_store_put.argtypes = [vp, vp, vp, u64]
    lib.ref_store_put.restype = ctypes.c_int64
    lib.ref_store_close.argtypes = [vp]
    lib.ref_store_close.restype = None
    lib.ref_store_get_plain.argtypes = [vp, vp, vp, u64, ctypes.POINTER(ctypes.c_double)]
    lib.ref_store_get_plain.restype = ctypes.c_int64
    lib.ref_store_get_probed.argtypes = [vp, vp, vp, u64, vp, vp, ctypes.POINTER(u64), ctypes.POINTER(ctypes.c_double)]
    lib.ref_store_get_probed.restype = ctypes.c_int64
    return lib


def reference_probe_fixture(data, offsets, n_put, n_query=None, max_slots=4096, folder=None):
    """Fill a store with the reference's own put (keys [0, n_put)), look up keys
    [0, n_query) with its own get, export its rows. Returns (uids, tab_slot,
    rows) as numpy arrays; uids[i] = the reference's shf_uid or 0xffffffff."""
    import tempfile
    import uuid

    lib = reference_lib()
    if lib is None:
        raise RuntimeError("oracle/_ref/libref_shf.so not built")
    data = np.ascontiguousarray(data).view(np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    if n_query is None:
        n_query = offsets.size - 1
    uids = np.empty(n_query, dtype=np.uint32)
    tab_slot = np.empty(256 * 2048, dtype=np.uint32)
    rows = np.zeros(max_slots * 65536, dtype=np.uint8)
    with tempfile.TemporaryDirectory(dir=folder or ("/dev/shm" if os.path.isdir("/dev/shm") else None)) as d:
        name = "probe" + uuid.uuid4().hex[:8]
        slots = lib.ref_probe_fixture(d.encode(), name.encode(), data.ctypes.data, offsets.ctypes.data, n_put,
                                      n_query, uids.ctypes.data, tab_slot.ctypes.data, rows.ctypes.data, max_slots)
    if slots < 0:
        raise RuntimeError("ref_probe_fixture failed (%d)" % slots)
    return uids, tab_slot, rows[: slots * 65536].copy()
