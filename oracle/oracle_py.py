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

# SHF_DATA_TYPE byte of copied records as the reference's build writes them
# (oracle/tab_oracle.h): 0x3e in shf_tab_shrink()'s copies, 0xbe in shf_tab_part()'s
TAB_KEEP_TYPE = 0x3E
TAB_MOVE_TYPE = 0xBE


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
        lib.oracle_tab_split.argtypes = [vp, u64, vp, u32, ctypes.c_int, u32, u32, u32, u32, u32, vp, u64, vp, u64]
        lib.oracle_tab_split.restype = ctypes.c_int
        lib.oracle_tab_part_redirect.argtypes = [vp, u32, u32]
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

    def tab_part_redirect(self, tab_map, tab_old, tab_new):
        """shf_tab_part()'s redirect of a window's 2048-entry tab2 -> tab map (a new array)."""
        m = np.array(tab_map, dtype=np.uint16)
        self.lib.oracle_tab_part_redirect(m.ctypes.data, tab_old, tab_new)
        return m

    def tab_split(self, src, tab_map, tab_new=0xFFFF, fixed=0, key_len=0, val_len=0, factor=1, cap=None,
                  keep_type=TAB_KEEP_TYPE, move_type=TAB_MOVE_TYPE):
        """(keep, move) tab images: the part/shrink copy of tab image `src`
        (tab_new = 0xFFFF: shrink only, move is None). keep_type / move_type:
        the data-type byte of the copies (oracle/tab_oracle.h)."""
        src = np.ascontiguousarray(src, dtype=np.uint8)
        m = np.ascontiguousarray(tab_map, dtype=np.uint16)
        cap = int(cap or src.size)
        keep = np.zeros(cap, dtype=np.uint8)
        move = np.zeros(cap, dtype=np.uint8) if tab_new != 0xFFFF else None
        rc = self.lib.oracle_tab_split(src.ctypes.data, src.size, m.ctypes.data, tab_new, int(fixed), key_len, val_len,
                                       factor, keep_type, move_type, keep.ctypes.data, cap,
                                       move.ctypes.data if move is not None else None, cap if move is not None else 0)
        if rc:
            raise ValueError("oracle_tab_split: output does not fit")
        return keep, move

    @staticmethod
    def win_order(hashes):
        """(perm, win_start): the key indices stably sorted by win = h1 & 0xff
        (shf.c:800), and each window's first position, then n (numpy)."""
        h = np.ascontiguousarray(hashes, dtype=np.uint64).reshape(-1, 2)
        win = (h[:, 0] & np.uint64(0xFF)).astype(np.int64)
        perm = np.argsort(win, kind="stable").astype(np.uint32)
        start = np.zeros(257, dtype=np.uint32)
        start[1:] = np.cumsum(np.bincount(win, minlength=256))
        return perm, start

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
    lib.ref_put_in_order.argtypes = [ctypes.c_char_p, ctypes.c_char_p, vp, vp, u64, vp, vp, vp, ctypes.c_int,
                                     ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
    lib.ref_put_in_order.restype = ctypes.c_int64
    lib.ref_put_get_procs.argtypes = [ctypes.c_char_p, ctypes.c_char_p, vp, vp, vp, vp, vp, ctypes.c_int, ctypes.c_int,
                                        ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
    lib.ref_put_get_procs.restype = ctypes.c_int64
    lib.ref_part_capture.argtypes = [ctypes.c_char_p, ctypes.c_char_p, vp, vp, u64, u32, u32, u32, u32,
                                     ctypes.c_char_p]
    lib.ref_part_capture.restype = ctypes.c_int64
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


def reference_part_capture(data, offsets, fixed_key_len=0, fixed_val_len=0, factor=1, max_caps=2, folder=None):
    """The reference's own shf_tab_part() (+ its shf_tab_shrink()), captured by
    oracle/ref_export.c ref_part_capture(): keys put one by one into a fresh
    store; for each put that parted a tab, the tab file before, both tab files
    after, and the window's tab map before/after. Returns a list of dicts."""
    import tempfile
    import uuid

    lib = reference_lib()
    if lib is None:
        raise RuntimeError("oracle/_ref/libref_shf.so not built")
    data = np.ascontiguousarray(data).view(np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = offsets.size - 1
    base = folder or ("/dev/shm" if os.path.isdir("/dev/shm") else None)
    with tempfile.TemporaryDirectory(dir=base) as store, tempfile.TemporaryDirectory(dir=base) as out:
        name = "part" + uuid.uuid4().hex[:8]
        caps = lib.ref_part_capture(store.encode(), name.encode(), data.ctypes.data, offsets.ctypes.data, n,
                                    fixed_key_len, fixed_val_len, factor, max_caps, out.encode())
        if caps < 0:
            raise RuntimeError("ref_part_capture failed (%d)" % caps)
        res = []
        for c in range(caps):
            rd = lambda ext: np.fromfile(os.path.join(out, "cap%d.%s" % (c, ext)), dtype=np.uint8)
            meta = rd("meta")
            m32 = meta[:36].view(np.uint32)
            maps = meta[36:].view(np.uint16)
            res.append({"win": int(m32[0]), "tab_old": int(m32[1]), "tab_new": int(m32[2]), "uid": int(m32[3]),
                        "key": int(m32[4]), "fixed": int(m32[5]), "fixed_key_len": int(m32[6]),
                        "fixed_val_len": int(m32[7]), "factor": int(m32[8]), "map_before": maps[:2048].copy(),
                        "map_after": maps[2048:].copy(), "before": rd("before"), "old": rd("old"),
                        "new": rd("new")})
        return res


def reference_put_in_order(data, offsets, hashes, order, folder, name, lockable=1):
    """The reference's own put loop over keys order[0..n) with the given hashes
    (oracle/ref_export.c ref_put_in_order), into a fresh store folder/name that
    stays on disk. order None = batch order. Returns (found, uids, put_seconds,
    get_seconds)."""
    lib = reference_lib()
    if lib is None:
        raise RuntimeError("oracle/_ref/libref_shf.so not built")
    data = np.ascontiguousarray(data).view(np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    hashes = np.ascontiguousarray(hashes, dtype=np.uint64)
    n = offsets.size - 1
    uids = np.zeros(n, dtype=np.uint32)
    order = None if order is None else np.ascontiguousarray(order, dtype=np.uint32)
    ps, gs = ctypes.c_double(), ctypes.c_double()
    found = lib.ref_put_in_order(folder.encode(), name.encode(), data.ctypes.data, offsets.ctypes.data, n,
                                 hashes.ctypes.data, order.ctypes.data if order is not None else None,
                                 uids.ctypes.data, lockable, ctypes.byref(ps), ctypes.byref(gs))
    if found < 0:
        raise RuntimeError("ref_put_in_order failed (%d)" % found)
    return found, uids, ps.value, gs.value


def store_files(folder, name):
    """{relative path: bytes} of every file of store folder/name (<name>.shf/...)."""
    root = os.path.join(folder, name + ".shf")
    out = {}
    for d, _, files in os.walk(root):
        for f in files:
            p = os.path.join(d, f)
            with open(p, "rb") as fh:
                out[os.path.relpath(p, root)] = fh.read()
    return out


def reference_put_get_procs(data, offsets, hashes, order, starts, folder, name, lockable=1):
    """The reference's put then get loops on len(starts) - 1 forked processes,
    process t over keys order[starts[t] .. starts[t+1]) (order None = batch
    order), each with its own handle on store folder/name (oracle/ref_export.c
    ref_put_get_procs). Call it from a process that has not touched the GPU.
    Returns (found, put_seconds, get_seconds)."""
    lib = reference_lib()
    if lib is None:
        raise RuntimeError("oracle/_ref/libref_shf.so not built")
    data = np.ascontiguousarray(data).view(np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    hashes = np.ascontiguousarray(hashes, dtype=np.uint64)
    starts = np.ascontiguousarray(starts, dtype=np.uint64)
    order = None if order is None else np.ascontiguousarray(order, dtype=np.uint32)
    ps, gs = ctypes.c_double(), ctypes.c_double()
    found = lib.ref_put_get_procs(folder.encode(), name.encode(), data.ctypes.data, offsets.ctypes.data,
                                    hashes.ctypes.data, order.ctypes.data if order is not None else None,
                                    starts.ctypes.data, starts.size - 1, lockable, ctypes.byref(ps), ctypes.byref(gs))
    if found < 0:
        raise RuntimeError("ref_put_get_procs failed (%d)" % found)
    return found, ps.value, gs.value
