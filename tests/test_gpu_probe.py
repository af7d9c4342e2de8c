"""Row pre-probe on the GPU: bit-exact against the oracle's
row scan (oracle_probe, pinned to the reference in tests/test_probe_oracle.py)
and against the reference's own get results, through the C ABI.
"""
import os

import numpy as np
import pytest

import sharedhashfile_amd as hb
from oracle.oracle_py import reference_lib, reference_probe_fixture
from sharedhashfile_amd.keygen import splitmix_bytes, splitmix_lengths
from sharedhashfile_amd.rowindex import synthetic_index

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "probe_fixture.npz")
NONE = 0xFFFFFFFF


@pytest.fixture(scope="module")
def torch():
    import torch

    assert torch.cuda.is_available()
    return torch


@pytest.fixture(scope="module")
def golden():
    with np.load(GOLDEN, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="module")
def golden_index(golden):
    idx = hb.RowIndex(golden["rows"].size // 65536, golden["tab_slot"], golden["rows"])
    yield idx
    idx.close()


def _u32(t):
    return t.cpu().numpy().view(np.uint32)


def _u64(t):
    return t.cpu().numpy().view(np.uint64)


def _dev(torch, a):
    a = np.ascontiguousarray(a)
    return torch.from_numpy(a if a.flags.writeable else a.copy()).cuda()


@pytest.mark.parametrize("kernel", [hb.KERNEL_AUTO, hb.KERNEL_FIXED16, hb.KERNEL_GENERIC, hb.KERNEL_SPAN])
def test_probe_fixture_every_kernel(torch, oracle, golden, golden_index, kernel):
    keys = _dev(torch, golden["keys"])
    rec, h = hb.probe_fixed(golden_index, keys, kernel=kernel, hashes=True)
    torch.cuda.synchronize()
    assert np.array_equal(_u64(h), golden["ref_hash"])
    want = oracle.probe(golden["ref_hash"], golden["tab_slot"], golden["rows"])
    assert np.array_equal(_u32(rec), want)
    n_put = int(golden["n_put"])
    assert np.array_equal(_u32(rec)[:n_put, 0], golden["ref_uid"][:n_put])  # = the reference's shf_uid


def test_probe_fixture_hashes_and_var_layout(torch, oracle, golden, golden_index):
    want = oracle.probe(golden["ref_hash"], golden["tab_slot"], golden["rows"])
    rec = hb.probe_hashes(golden_index, _dev(torch, golden["ref_hash"].view(np.int64)))
    torch.cuda.synchronize()
    assert np.array_equal(_u32(rec), want)
    n = golden["keys"].shape[0]
    off = _dev(torch, (np.arange(n + 1, dtype=np.int64) * 16))
    rec2 = hb.probe_var(golden_index, _dev(torch, golden["keys"].reshape(-1)), off)
    torch.cuda.synchronize()
    assert np.array_equal(_u32(rec2), want)


@pytest.mark.skipif(reference_lib() is None, reason="oracle/_ref not built")
def test_probe_var_keys_against_reference_store(torch, oracle):
    n = 60000
    lens = splitmix_lengths(n, 1, 400, 21)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    data = np.frombuffer(splitmix_bytes(int(off[-1]), 22), dtype=np.uint8)
    n_put = 50000
    uids, tab_slot, rows = reference_probe_fixture(data, off, n_put)
    idx = hb.RowIndex(rows.size // 65536, tab_slot, rows)
    try:
        rec, h = hb.probe_var(idx, _dev(torch, data), _dev(torch, off.view(np.int64)), hashes=True)
        torch.cuda.synchronize()
        hh = oracle.hash_var(data, off)
        assert np.array_equal(_u64(h), hh)
        got = _u32(rec)
        assert np.array_equal(got, oracle.probe(hh, tab_slot, rows))
        found = uids != NONE
        # short keys can repeat; where the reference found the key, the row scan must list its ref
        mask = got[:, 2] & 0xFFFF
        assert ((mask[found] >> ((uids[found] >> 28) & 15)) & 1).all()
        single = np.array([bin(int(m)).count("1") == 1 for m in mask])
        assert np.array_equal(got[found & single, 0], uids[found & single])
    finally:
        idx.close()


@pytest.mark.parametrize("key_len,kernel", [(16, hb.KERNEL_FIXED16), (37, hb.KERNEL_GENERIC),
                                            (100, hb.KERNEL_SPAN), (256, hb.KERNEL_TILED),
                                            (192, hb.KERNEL_TILED), (64, hb.KERNEL_AUTO)])
def test_probe_synthetic_index_all_kernels(torch, oracle, key_len, kernel):
    n = 300_000
    keys = np.frombuffer(splitmix_bytes(n * key_len, 40 + key_len), dtype=np.uint8).reshape(n, key_len)
    h = oracle.hash_fixed(keys, threads=8)
    tab_slot, rows, n_slots, placed = synthetic_index(h, tabs_per_win=2, limit=n * 3 // 4)
    idx = hb.RowIndex(n_slots, tab_slot, rows)
    try:
        rec, hh = hb.probe_fixed(idx, _dev(torch, keys), kernel=kernel, hashes=True)
        torch.cuda.synchronize()
        assert np.array_equal(_u64(hh), h)
        want = oracle.probe(h, tab_slot, rows)
        assert np.array_equal(_u32(rec), want)
        assert (want[: n * 3 // 4, 0] != NONE).mean() > 0.999
    finally:
        idx.close()


def test_probe_ragged_index(torch, oracle):
    """Entries naming slots past n_slots, unindexed windows, an empty index."""
    n = 50_000
    keys = np.frombuffer(splitmix_bytes(n * 24, 77), dtype=np.uint8).reshape(n, 24)
    h = oracle.hash_fixed(keys)
    tab_slot, rows, n_slots, _ = synthetic_index(h, tabs_per_win=4)
    tab_slot = tab_slot.copy()
    tab_slot[: 2048 * 16] = NONE  # windows 0..15 unindexed
    short = n_slots - 300  # the last 300 slots are missing from the index
    idx = hb.RowIndex(short, tab_slot, rows[: short * 65536])
    empty = hb.RowIndex(0, np.full(256 * 2048, NONE, dtype=np.uint32))
    try:
        d = _dev(torch, keys)
        rec = hb.probe_fixed(idx, d)
        rec0 = hb.probe_fixed(empty, d)
        torch.cuda.synchronize()
        assert np.array_equal(_u32(rec), oracle.probe(h, tab_slot, rows[: short * 65536], n_slots=short))
        r0 = _u32(rec0)
        assert (r0[:, 0] == NONE).all() and (r0[:, 2] == 0xFFFF << 16).all() and (r0[:, 3] == NONE).all()
    finally:
        idx.close()
        empty.close()


def test_probe_compact_map_ranks_escapes_and_device_writes(torch, oracle):
    """The probes read a compact copy of tab_slot that set_tabs makes (a rank per
    entry among its window's distinct entries + the windows' entry lists). Windows
    with 254 distinct entries (every rank used), 255 (one escape to tab_slot) and
    2048 (mostly escapes), then writes through the device pointers, which the
    probes must see at once (they then read tab_slot itself)."""
    import ctypes

    n = 200_000
    keys = np.frombuffer(splitmix_bytes(n * 16, 91), dtype=np.uint8).reshape(n, 16)
    h = oracle.hash_fixed(keys)
    tab_slot, rows, n_slots, _ = synthetic_index(h, tabs_per_win=2)
    ts = tab_slot.copy().reshape(256, 2048)
    slot = ts >> np.uint32(11)
    t2 = np.arange(2048, dtype=np.uint32)
    ts[0] = (slot[0] << np.uint32(11)) | t2                      # 2048 distinct: ranks 0..253, then escapes
    ts[1] = (slot[1] << np.uint32(11)) | (t2 % np.uint32(254))   # exactly 254 distinct
    ts[2] = (slot[2] << np.uint32(11)) | (t2 % np.uint32(255))   # 255: one value escapes
    ts[3, ::3] = NONE                                            # some entries unindexed
    ts = ts.reshape(-1)
    idx = hb.RowIndex(n_slots, ts, rows)
    try:
        d = _dev(torch, keys)
        for kernel in (hb.KERNEL_FIXED16, hb.KERNEL_GENERIC):
            rec = hb.probe_fixed(idx, d, kernel=kernel)
            torch.cuda.synchronize()
            assert np.array_equal(_u32(rec), oracle.probe(h, ts, rows)), kernel
        # writes through the device pointers (a producer filling the index on the device)
        d_ts, _, _ = idx.device_ptrs()
        ts2 = ts.copy().reshape(256, 2048)
        ts2[4:8] = NONE
        ts2[9] = ts2[10]
        ts2 = ts2.reshape(-1)
        src = torch.from_numpy(ts2.view(np.int32)).to("cuda")
        hip = ctypes.CDLL("libamdhip64.so")
        hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        torch.cuda.synchronize()
        assert hip.hipMemcpy(d_ts, src.data_ptr(), ts2.nbytes, 3) == 0  # hipMemcpyDeviceToDevice
        rec = hb.probe_fixed(idx, d)
        torch.cuda.synchronize()
        assert np.array_equal(_u32(rec), oracle.probe(h, ts2, rows))
    finally:
        idx.close()


def test_probe_full_size_config_b(torch, oracle):
    """configs[1] shape (10M x 16 B) with a device-built index: GPU hashes and
    probes agree across kernels; a 20 000-key sample agrees with the oracle."""
    from sharedhashfile_amd.keygen import device_random_bytes

    n = 10_000_000
    keys = device_random_bytes(n * 16, seed=5, device="cuda").view(n, 16)
    h = hb.hash_fixed(keys)
    tab_slot, rows, n_slots, placed = synthetic_index(h, tabs_per_win=16, limit=n // 2)
    idx = hb.RowIndex(n_slots, tab_slot, rows)  # device tensors: copied on the device
    try:
        rec_a = hb.probe_fixed(idx, keys)
        rec_b = hb.probe_fixed(idx, keys, kernel=hb.KERNEL_GENERIC)
        rec_c = hb.probe_hashes(idx, h)
        torch.cuda.synchronize()
        assert torch.equal(rec_a, rec_b) and torch.equal(rec_a, rec_c)
        sample = np.linspace(0, n - 1, 20000).astype(np.int64)
        hs = _u64(h)[sample]
        ts_np = tab_slot.cpu().numpy().view(np.uint32)
        rows_np = rows.cpu().numpy()
        assert np.array_equal(_u32(rec_a)[sample], oracle.probe(hs, ts_np, rows_np))
        hit = _u32(rec_a)[:, 0] != NONE
        assert hit[: n // 2].mean() > 0.999 and hit[n // 2:].mean() < 0.001
    finally:
        idx.close()



@pytest.mark.skipif(reference_lib() is None, reason="oracle/_ref not built")
def test_probe_drives_reference_get(torch, tmp_path_factory):
    """f3 end to end: the reference fills a store; its rows go to HBM; the GPU
    hashes and probes a get batch; the reference's get then serves every stored
    key through the probe's uid (shf_get_uid_val_copy + key compare) with the
    right value, and falls back to its ordinary get for the rest."""
    import ctypes
    import tempfile
    import time

    lib = reference_lib()
    n_put, n_abs = 200_000, 20_000
    n = n_put + n_abs
    lens = splitmix_lengths(n, 8, 200, 31)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    data = np.frombuffer(splitmix_bytes(int(off[-1]), 32), dtype=np.uint8)
    with tempfile.TemporaryDirectory(dir="/dev/shm" if os.path.isdir("/dev/shm") else None) as d:
        shf = lib.ref_store_open(d.encode(), b"probe_get")
        assert shf
        try:
            assert lib.ref_store_put(shf, data.ctypes.data, off.ctypes.data, n_put) == n_put
            ts = np.empty(256 * 2048, dtype=np.uint32)
            rows = np.zeros(4096 * 65536, dtype=np.uint8)
            slots = lib.ref_export_rows(shf, ts.ctypes.data, rows.ctypes.data, 4096)
            assert slots >= 256
            idx = hb.RowIndex(slots, ts, rows[: slots * 65536])
            t0 = time.perf_counter()
            rec, h = hb.probe_var(idx, _dev(torch, data), _dev(torch, off.view(np.int64)), hashes=True)
            torch.cuda.synchronize()
            gpu_s = time.perf_counter() - t0
            rec_np, h_np = _u32(rec), _u64(h)
            fast, sec = ctypes.c_uint64(), ctypes.c_double()
            good = lib.ref_store_get_probed(shf, data.ctypes.data, off.ctypes.data, n, rec_np.ctypes.data,
                                            h_np.ctypes.data, ctypes.byref(fast), ctypes.byref(sec))
            assert good == n_put and fast.value == n_put
            sec_plain = ctypes.c_double()
            assert lib.ref_store_get_plain(shf, data.ctypes.data, off.ctypes.data, n, ctypes.byref(sec_plain)) == n_put
            print("get loop: reference %.1f ns/key, probe-driven %.1f ns/key (+ GPU %.1f ms incl. copies)" % (
                1e9 * sec_plain.value / n, 1e9 * sec.value / n, 1e3 * gpu_s))
            idx.close()
        finally:
            lib.ref_store_close(shf)


def test_probe_host_memory_paths(torch, oracle, golden, golden_index):
    """shf_probe_batch_fixed / _var with host buffers (pipelined through pinned
    staging) and with device buffers (synchronous)."""
    want = oracle.probe(golden["ref_hash"], golden["tab_slot"], golden["rows"])
    rec, h = hb.probe_fixed_host(golden_index, golden["keys"], hashes=True)
    assert np.array_equal(rec, want) and np.array_equal(h, golden["ref_hash"])
    n = golden["keys"].shape[0]
    off = np.arange(n + 1, dtype=np.uint64) * 16
    assert np.array_equal(hb.probe_var_host(golden_index, golden["keys"].reshape(-1), off), want)
    lib = hb.load()
    d_keys = _dev(torch, golden["keys"])
    d_rec = torch.empty((n, 4), dtype=torch.int32, device="cuda")
    assert lib.shf_probe_batch_fixed(golden_index.handle, d_keys.data_ptr(), 16, n, hb.SEED, None,
                                     d_rec.data_ptr(), hb.MEM_DEVICE) == hb.OK
    assert np.array_equal(_u32(d_rec), want)


def test_probe_host_multi_chunk_var(torch, oracle):
    """More key bytes than one 64 MiB staging chunk, variable lengths, pinned
    output buffers (DMA'd straight into) and pageable ones."""
    n = 400_000
    lens = splitmix_lengths(n, 100, 400, 61)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)  # ~100 MB
    data = np.frombuffer(splitmix_bytes(int(off[-1]), 62), dtype=np.uint8)
    h = oracle.hash_var(data, off)
    tab_slot, rows, n_slots, _ = synthetic_index(h, tabs_per_win=2, limit=n - 1000)
    idx = hb.RowIndex(n_slots, tab_slot, rows)
    try:
        want = oracle.probe(h, tab_slot, rows)
        rec, hh = hb.probe_var_host(idx, data, off, hashes=True)
        assert np.array_equal(rec, want) and np.array_equal(hh, h)
        lib = hb.load()
        p_rec = torch.zeros((n, 4), dtype=torch.int32).pin_memory()
        p_h = torch.zeros((n, 2), dtype=torch.int64).pin_memory()
        assert lib.shf_probe_batch_var(idx.handle, data.ctypes.data, off.ctypes.data, n, hb.SEED, p_h.data_ptr(),
                                       p_rec.data_ptr(), hb.MEM_HOST) == hb.OK
        assert np.array_equal(p_rec.numpy().view(np.uint32), want)
        assert np.array_equal(p_h.numpy().view(np.uint64), h)
    finally:
        idx.close()
