"""Drop-in check against the reference's own table engine.

Hashes made by the GPU batch path re-enter the reference's unchanged
put/get/del flow through its caller-supplied-hash seam
(/root/reference/src/test.9.shf.c:176-182): set shf_hash / shf_hash_key /
shf_hash_key_len, then shf_put_key_val(). Every key is then read back through
the reference's own shf_make_hash() + shf_get_key_val_copy() (and the other way
round). Any hash that differs from the reference's in the 49 bits put/find use
(shf.c:800-803, :893-896) would put the key where the reference cannot find it.

The reference code here is oracle/_ref/libref_shf.so (reference src/shf.c +
murmurhash3.c + oracle/ref_harness.c), test infrastructure only.
"""
import ctypes
import os

import numpy as np
import pytest

from oracle.oracle_py import REF_SO


def _ref():
    if not os.path.exists(REF_SO):
        pytest.skip("oracle/_ref/libref_shf.so not built")
    lib = ctypes.CDLL(REF_SO)
    lib.ref_roundtrip_with_hashes.restype = ctypes.c_int64
    lib.ref_roundtrip_with_hashes.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int]
    return lib


def _unique_keys(n, seed, lo=4, hi=300):
    """n distinct variable-length keys: 4-byte LE index prefix + random bytes."""
    rng = np.random.default_rng(seed)
    lens = rng.integers(lo, hi + 1, size=n)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    data = rng.integers(0, 256, size=int(off[-1]), dtype=np.uint8)
    idx = np.arange(n, dtype="<u4").view(np.uint8).reshape(n, 4)
    starts = off[:-1].astype(np.int64)
    for b in range(4):
        data[starts + b] = idx[:, b]
    return data, off


def _roundtrip(lib, data, off, hashes, mode):
    name = ("shfhb-%d-%d" % (os.getpid(), mode)).encode()
    hashes = np.ascontiguousarray(hashes, dtype=np.uint64)
    return lib.ref_roundtrip_with_hashes(b"/dev/shm", name, data.ctypes.data, off.ctypes.data, off.size - 1,
                                         hashes.ctypes.data, mode)


def test_harness_with_oracle_hashes(oracle):
    lib = _ref()
    data, off = _unique_keys(20000, 1)
    h = oracle.hash_var(data, off)
    assert _roundtrip(lib, data, off, h, 0) == 20000
    assert _roundtrip(lib, data, off, h, 1) == 20000
    bad = h.copy()
    bad[::2, 0] ^= np.uint64(1 << 5)  # flips a `win` bit of every other key
    assert _roundtrip(lib, data, off, bad, 0) < 15000


@pytest.mark.gpu
def test_gpu_hashes_drop_into_reference_put_get(hb):
    lib = _ref()
    data, off = _unique_keys(200000, 2)
    h = hb.hash_var_host(data, off)  # GPU, host-memory entry point
    assert _roundtrip(lib, data, off, h, 0) == 200000
    assert _roundtrip(lib, data, off, h, 1) == 200000
    # fixed 16-byte keys through the fixed-length entry point
    n = 100000
    keys = np.zeros((n, 16), dtype=np.uint8)
    keys[:, :4] = np.arange(n, dtype="<u4").view(np.uint8).reshape(n, 4)
    keys[:, 4:] = np.random.default_rng(3).integers(0, 256, size=(n, 12), dtype=np.uint8)
    h16 = hb.hash_fixed_host(keys, 16)
    off16 = np.arange(n + 1, dtype=np.uint64) * 16
    assert _roundtrip(lib, keys.reshape(-1), off16, h16, 0) == n
