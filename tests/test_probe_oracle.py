"""Row pre-probe, CPU side: the oracle's row scan pinned to
the reference's own put/get, and the synthetic index generator.

The oracle (oracle_probe, oracle/murmur3_oracle.c) restates the row scan of
shf_find_key_internal() (/root/reference/src/shf.c:886-922). Pinning:
  * tests/golden/probe_fixture.npz: a store filled and queried by the
    reference itself (tests/golden/make_probe_golden.py), including a parted
    window;
  * where oracle/_ref is built: a fresh store with variable-length keys,
    filled and queried by the reference in this process.
"""
import os

import numpy as np
import pytest

from oracle.oracle_py import reference_lib, reference_probe_fixture
from sharedhashfile_amd.keygen import splitmix_bytes, splitmix_lengths
from sharedhashfile_amd.rowindex import synthetic_index

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "probe_fixture.npz")
NONE = 0xFFFFFFFF


@pytest.fixture(scope="module")
def probe_golden():
    with np.load(GOLDEN, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def _popcount16(m):
    m = m.astype(np.uint32)
    return np.array([bin(int(x)).count("1") for x in m])


def test_fixture_hashes_are_the_oracles(oracle, probe_golden):
    g = probe_golden
    assert np.array_equal(oracle.hash_fixed(g["keys"]), g["ref_hash"])


def test_oracle_probe_matches_reference_get(oracle, probe_golden):
    g = probe_golden
    n_put = int(g["n_put"])
    rec = oracle.probe(g["ref_hash"], g["tab_slot"], g["rows"])
    uid = g["ref_uid"]
    # every stored key: the first candidate is the ref the reference's get found
    assert np.array_equal(rec[:n_put, 0], uid[:n_put])
    mask = rec[:, 2] & 0xFFFF
    assert (_popcount16(mask[:n_put]) >= 1).all()
    # pos points at a record (non-zero) and the physical tab is the slot's
    assert (rec[:n_put, 1] != 0).all()
    ts = g["tab_slot"]
    win = g["ref_hash"][:, 0] & 0xFF
    tab2 = (g["ref_hash"][:, 0] >> 16) & 0x7FF
    e = ts[(win << 11) | tab2]
    assert np.array_equal(rec[:, 3], e >> 11)
    assert np.array_equal(rec[:, 2] >> 16, e & 0x7FF)
    # keys never put: no candidate, uid NONE (as the reference's get: not found)
    assert (uid[n_put:] == NONE).all()
    assert (rec[n_put:, 0] == NONE).all() and (mask[n_put:] == 0).all()
    # window 0 was parted: its tab2s map to more than one physical tab
    assert len(set((ts[:2048] & 0x7FF).tolist())) > 1


def test_oracle_probe_row_semantics(oracle):
    """Hand-built rows: pos == 0 never matches, tab and rnd must both match,
    the first candidate in ref order wins, unindexed tabs are absent."""
    h1 = (0x0123 << 32) | (0x0456 << 16) | 0x07  # win 7, tab2 0x456, row 0x123
    h2 = 0x1ABCDE  # rnd
    hashes = np.array([[h1, h2]], dtype=np.uint64)
    win, tab2, row, rnd = 7, 0x456, 0x123, 0x1ABCDE
    tab_slot = np.full(256 * 2048, NONE, dtype=np.uint32)
    tab_slot[(win << 11) | tab2] = (1 << 11) | 5  # slot 1, physical tab 5
    rows = np.zeros(2 * 65536, dtype=np.uint8)
    refs = rows.view(np.uint32).reshape(2, 512, 16, 2)
    want = tab2 | (rnd << 11)
    refs[1, row, 0] = (want, 0)  # matches but unused
    refs[1, row, 1] = (want ^ 1, 11)  # tab mismatch
    refs[1, row, 2] = (want ^ (1 << 11), 12)  # rnd mismatch
    refs[1, row, 5] = (want, 99)  # first candidate
    refs[1, row, 9] = (want, 77)  # second candidate
    rec = oracle.probe(hashes, tab_slot, rows)[0]
    assert rec[0] == win | (tab2 << 8) | (row << 19) | (5 << 28)
    assert rec[1] == 99
    assert rec[2] == ((1 << 5) | (1 << 9)) | (5 << 16)
    assert rec[3] == 1
    # a slot past n_slots and an unindexed tab are both "absent"
    assert tuple(oracle.probe(hashes, tab_slot, rows, n_slots=1)[0]) == (NONE, 0, 0xFFFF << 16, NONE)
    tab_slot[(win << 11) | tab2] = NONE
    assert tuple(oracle.probe(hashes, tab_slot, rows)[0]) == (NONE, 0, 0xFFFF << 16, NONE)


@pytest.mark.skipif(reference_lib() is None, reason="oracle/_ref not built")
def test_oracle_probe_matches_reference_var_keys(oracle):
    n = 40000
    lens = splitmix_lengths(n, 8, 300, 7)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    data = np.frombuffer(splitmix_bytes(int(off[-1]), 8), dtype=np.uint8)
    n_put = 36000
    uids, tab_slot, rows = reference_probe_fixture(data, off, n_put)
    rec = oracle.probe(oracle.hash_var(data, off), tab_slot, rows)
    found = uids != NONE
    assert found[:n_put].all() and not found[n_put:].any()
    assert np.array_equal(rec[:n_put, 0], uids[:n_put])
    assert (rec[n_put:, 0] == NONE).all()


def test_synthetic_index_numpy_finds_every_placed_key(oracle):
    keys = np.frombuffer(splitmix_bytes(50000 * 16, 3), dtype=np.uint8).reshape(-1, 16)
    h = oracle.hash_fixed(keys)
    tab_slot, rows, n_slots, placed = synthetic_index(h, tabs_per_win=2, limit=45000)
    assert placed == 45000 and n_slots == 512
    rec = oracle.probe(h, tab_slot, rows)
    pos = np.arange(1, 50001, dtype=np.uint32)
    hit = rec[:, 0] != NONE
    assert hit[:45000].all()
    assert (rec[:45000, 1] == pos[:45000]).mean() > 0.999  # rnd collisions inside a row are rare
    assert hit[45000:].sum() <= 2


def test_synthetic_index_torch_equals_numpy(oracle):
    import torch

    keys = np.frombuffer(splitmix_bytes(20000 * 16, 4), dtype=np.uint8).reshape(-1, 16)
    h = oracle.hash_fixed(keys)
    a = synthetic_index(h, tabs_per_win=3)
    b = synthetic_index(torch.from_numpy(h.view(np.int64)), tabs_per_win=3)
    assert np.array_equal(a[0], b[0].numpy().view(np.uint32))
    assert np.array_equal(a[1], b[1].numpy())
    assert a[2:] == b[2:]


@pytest.mark.skipif(reference_lib() is None, reason="oracle/_ref not built")
def test_probe_records_drive_reference_get(oracle):
    """The INTEGRATION.md §6 get loop on the reference's own store, fed with
    oracle probe records (tests/test_gpu_probe.py feeds it the GPU's)."""
    import ctypes
    import tempfile

    lib = reference_lib()
    n_put, n_abs = 30_000, 5_000
    n = n_put + n_abs
    lens = splitmix_lengths(n, 8, 120, 41)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    data = np.frombuffer(splitmix_bytes(int(off[-1]), 42), dtype=np.uint8)
    with tempfile.TemporaryDirectory(dir="/dev/shm" if os.path.isdir("/dev/shm") else None) as d:
        shf = lib.ref_store_open(d.encode(), b"probe_get_cpu")
        assert shf
        try:
            assert lib.ref_store_put(shf, data.ctypes.data, off.ctypes.data, n_put) == n_put
            ts = np.empty(256 * 2048, dtype=np.uint32)
            rows = np.zeros(1024 * 65536, dtype=np.uint8)
            slots = lib.ref_export_rows(shf, ts.ctypes.data, rows.ctypes.data, 1024)
            assert slots >= 256
            h = oracle.hash_var(data, off)
            rec = oracle.probe(h, ts, rows[: slots * 65536])
            fast, sec = ctypes.c_uint64(), ctypes.c_double()
            good = lib.ref_store_get_probed(shf, data.ctypes.data, off.ctypes.data, n, rec.ctypes.data, h.ctypes.data,
                                            ctypes.byref(fast), ctypes.byref(sec))
            assert good == n_put and fast.value == n_put
            # a stale probe (candidate uid pointing at another key) is caught by the key compare
            bad = rec.copy()
            bad[:n_put:2] = rec[1:n_put:2][: bad[:n_put:2].shape[0]]
            good2 = lib.ref_store_get_probed(shf, data.ctypes.data, off.ctypes.data, n, bad.ctypes.data,
                                             h.ctypes.data, ctypes.byref(fast), ctypes.byref(sec))
            assert good2 == n_put and fast.value < n_put
        finally:
            lib.ref_store_close(shf)
