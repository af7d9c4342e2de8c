"""UID parts from host memory (shf_uid_parts_batch_fixed / _var, SHF_HASH_MEM_HOST).

The reference's put and find read 49 bits of each key's hash: win, tab2, row
and rnd (/root/reference/src/shf.c:800-803, :893-896). The UID-parts calls
return exactly those, packed in 8 B per key (include/shf_hash_batch.h
SHF_UID_PARTS_*), so a host caller moves 8 B per key back over PCIe instead of
16. The seam side -- shf_use_uid_parts() rebuilding the SHF_HASH fields the
reference reads, and a store put that way ending byte-equal to a full-hash put
-- is tests/c/test_seam.c section 7 (tests/test_c_seam.py).

Parity: against oracle.uid_parts(oracle.hash_*) (oracle/, pinned to the
reference by tests/test_oracle.py), exactly at up to 10M keys, and at
BASELINE configs[4]'s 1B x 16 B against the device kernels for every key plus
an oracle sample.
"""
import numpy as np
import pytest

from sharedhashfile_amd.keygen import device_random_bytes, splitmix_bytes

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev(hb):
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    hb.check_device()
    return torch.device("cuda:0")


def _want_fixed(oracle, flat, L):
    return oracle.uid_parts(oracle.hash_fixed(flat, L, threads=8))


@pytest.mark.parametrize("key_len", [0, 1, 4, 15, 16, 17, 32, 100, 256, 511])
def test_host_uid_fixed_lengths(hb, dev, oracle, key_len):
    n = 70_001
    flat = np.frombuffer(splitmix_bytes(n * key_len + 1, 300 + key_len), dtype=np.uint8)[: n * key_len]
    if key_len:
        assert np.array_equal(hb.uid_parts_fixed_host(flat, key_len), _want_fixed(oracle, flat, key_len))
        return
    # zero-length keys (no key bytes at all): every key's parts are those of the empty key
    out = np.zeros(n, dtype=np.uint64)
    assert hb.load().shf_uid_parts_batch_fixed(None, 0, n, 12345, out.ctypes.data, hb.MEM_HOST) == 0
    empty = oracle.uid_parts(oracle.hash_var(np.zeros(1, np.uint8), np.zeros(2, np.uint64)))[0]
    assert np.all(out == empty)


@pytest.mark.parametrize("stage_mb,slots,pool_mb", [(1, 2, 64), (1, 4, 1), (3, 3, 64), (16, 4, 64)])
def test_host_uid_pipeline_shapes(hb, dev, oracle, monkeypatch, stage_mb, slots, pool_mb):
    """Many chunks (8-B records: more keys per slot than with hashes), a pool of
    one slot, and a variable-length key larger than a slot."""
    monkeypatch.setenv("SHF_HB_STAGE_MB", str(stage_mb))
    monkeypatch.setenv("SHF_HB_SLOTS", str(slots))
    monkeypatch.setenv("SHF_HB_POOL_MB", str(pool_mb))
    n = 900_000
    flat = np.frombuffer(splitmix_bytes(n * 16, 310 + stage_mb), dtype=np.uint8)
    assert np.array_equal(hb.uid_parts_fixed_host(flat, 16), _want_fixed(oracle, flat, 16))
    rng = np.random.default_rng(311 + slots)
    m = 30_000
    lens = rng.integers(0, 700, size=m)
    lens[7] = 3 << 20
    off = np.zeros(m + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    data = rng.integers(0, 256, size=int(off[-1]), dtype=np.uint8)
    assert np.array_equal(hb.uid_parts_var_host(data, off), oracle.uid_parts(oracle.hash_var(data, off)))


@pytest.mark.parametrize("direct_out", ["1", "0"])
@pytest.mark.parametrize("zero_copy", ["128", "0"])
def test_host_uid_pinned(hb, dev, oracle, monkeypatch, direct_out, zero_copy):
    """Page-locked caller buffers: the kernel reads the keys and writes the parts
    over PCIe (zero copy), or both go through the copy engines, the parts stored
    by the kernel into the caller's page-locked output or copied back per chunk."""
    monkeypatch.setenv("SHF_HB_DIRECT_OUT", direct_out)
    monkeypatch.setenv("SHF_HB_ZERO_COPY_MAX_KEY", zero_copy)
    lib = hb.load()
    n, pad = 2_000_003, 3
    keys = torch.randint(0, 256, (n * 16 + pad,), dtype=torch.uint8).pin_memory()
    out = torch.zeros(n + 1, dtype=torch.int64).pin_memory()
    rc = lib.shf_uid_parts_batch_fixed(keys.data_ptr() + pad, 16, n, 12345, out.data_ptr() + 8, hb.MEM_HOST)
    assert rc == 0
    assert out[0].item() == 0
    assert np.array_equal(out.numpy().view(np.uint64)[1:], _want_fixed(oracle, keys.numpy()[pad:], 16))
    m = 150_000
    lens = np.random.default_rng(33).integers(0, 600, size=m)
    off = torch.zeros(m + 1, dtype=torch.int64).pin_memory()
    off[1:] = torch.from_numpy(np.cumsum(lens))
    data = torch.randint(0, 256, (int(off[-1]),), dtype=torch.uint8).pin_memory()
    out2 = torch.zeros(m, dtype=torch.int64).pin_memory()
    rc = lib.shf_uid_parts_batch_var(data.data_ptr(), off.data_ptr(), m, 12345, out2.data_ptr(), hb.MEM_HOST)
    assert rc == 0
    want = oracle.uid_parts(oracle.hash_var(data.numpy(), off.numpy().view(np.uint64)))
    assert np.array_equal(out2.numpy().view(np.uint64), want)


def test_uid_sync_device_memory(hb, dev, oracle):
    """mem = SHF_HASH_MEM_DEVICE: the synchronous forms on HBM buffers (after the
    caller's null-stream work, as the hashing calls)."""
    lib = hb.load()
    n = 500_000
    keys = torch.randint(0, 256, (n * 24,), dtype=torch.uint8, device=dev)
    out = torch.empty(n, dtype=torch.int64, device=dev)
    assert lib.shf_uid_parts_batch_fixed(keys.data_ptr(), 24, n, 12345, out.data_ptr(), hb.MEM_DEVICE) == 0
    assert np.array_equal(out.cpu().numpy().view(np.uint64), _want_fixed(oracle, keys.cpu().numpy(), 24))
    lens = torch.randint(0, 300, (n,), device=dev)
    off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    torch.cumsum(lens, 0, out=off[1:])
    data = torch.randint(0, 256, (int(off[-1].item()),), dtype=torch.uint8, device=dev)
    assert lib.shf_uid_parts_batch_var(data.data_ptr(), off.data_ptr(), n, 12345, out.data_ptr(), hb.MEM_DEVICE) == 0
    want = oracle.uid_parts(oracle.hash_var(data.cpu().numpy(), off.cpu().numpy().view(np.uint64)))
    assert np.array_equal(out.cpu().numpy().view(np.uint64), want)
    # a decreasing offset: SHF_HB_ERR_ARG, every valid key still written
    off[5] = off[4] - 1
    out.fill_(0)
    assert lib.shf_uid_parts_batch_var(data.data_ptr(), off.data_ptr(), n, 12345, out.data_ptr(),
                                       hb.MEM_DEVICE) == hb.ERR_ARG


def test_host_uid_bad_arguments(hb, dev):
    lib = hb.load()
    out = np.zeros(4, dtype=np.uint64)
    keys = np.zeros(64, dtype=np.uint8)
    assert lib.shf_uid_parts_batch_fixed(keys.ctypes.data, 16, 4, 12345, None, hb.MEM_HOST) == hb.ERR_ARG
    assert lib.shf_uid_parts_batch_fixed(keys.ctypes.data, 16, 4, 12345, out.ctypes.data, 7) == hb.ERR_ARG
    assert lib.shf_uid_parts_batch_fixed(keys.ctypes.data, 0x80000000, 4, 12345, out.ctypes.data,
                                         hb.MEM_HOST) == hb.ERR_ARG
    off = np.array([0, 8, 4, 12, 16], dtype=np.uint64)  # decreasing: refused before any copy
    out[:] = 7
    assert lib.shf_uid_parts_batch_var(keys.ctypes.data, off.ctypes.data, 4, 12345, out.ctypes.data,
                                       hb.MEM_HOST) == hb.ERR_ARG
    assert np.all(out == 7)
    assert lib.shf_uid_parts_batch_fixed(keys.ctypes.data, 16, 0, 12345, None, hb.MEM_HOST) == 0  # n = 0


def test_host_uid_10m_16b_exact(hb, dev, oracle):
    """BASELINE configs[1]'s 10M x 16 B from pageable buffers: every key's parts
    against the oracle, and against the parts of the 16-B host hashes."""
    n = 10_000_000
    flat = device_random_bytes(n * 16, 320, dev).cpu().numpy()
    got = hb.uid_parts_fixed_host(flat, 16)
    assert np.array_equal(got, _want_fixed(oracle, flat, 16))
    assert np.array_equal(got, oracle.uid_parts(hb.hash_fixed_host(flat, 16)))


def test_host_uid_config3_10m_var(hb, dev, oracle):
    """configs[3]'s U[8,512] B keys, 10M of them from pageable buffers: every
    key against the device kernel's parts, and against the oracle."""
    n = 10_000_000
    g = torch.Generator(device=dev)
    g.manual_seed(321)
    lens = torch.randint(8, 513, (n,), generator=g, device=dev, dtype=torch.int64)
    off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    torch.cumsum(lens, 0, out=off[1:])
    del lens
    data = device_random_bytes(int(off[-1].item()), 322, dev)
    ref = hb.uid_parts_var(data, off).cpu().numpy().view(np.uint64)
    h_data, h_off = data.cpu().numpy(), off.cpu().numpy().view(np.uint64)
    del data, off
    got = hb.uid_parts_var_host(h_data, h_off)
    assert np.array_equal(got, ref)
    assert np.array_equal(got, oracle.uid_parts(oracle.hash_var(h_data, h_off)))


def test_host_uid_config4_1b_16b(hb, dev, oracle):
    """BASELINE configs[4]'s 1B x 16 B (16 GB of keys) from pageable buffers:
    every key against the device kernel's parts (compared on the device), a
    sample against the oracle."""
    n = 1_000_000_000
    keys = device_random_bytes(n * 16, 323, dev)
    ref = hb.uid_parts_fixed(keys, 16)
    host = keys.cpu().numpy()
    del keys
    got = hb.uid_parts_fixed_host(host, 16)
    assert torch.equal(torch.from_numpy(got.view(np.int64)).to(dev), ref)
    del ref
    idx = np.unique(np.concatenate([np.random.default_rng(323).integers(0, n, size=20000), [0, n - 1]]))
    assert np.array_equal(got[idx], _want_fixed(oracle, host.reshape(n, 16)[idx], 16))


@pytest.mark.parametrize("n_devices", [0, 3, 8])
def test_host_uid_multi(hb, dev, oracle, monkeypatch, n_devices):
    """shf_uid_parts_batch_{fixed,var}_multi: the host batch split over shard
    threads (here sharing this GPU: SHF_HB_MULTI_SHARE_DEVICES; 0 = every
    visible device), every key's parts as one call makes them."""
    monkeypatch.setenv("SHF_HB_MULTI_SHARE_DEVICES", "1")
    n = 3_000_017
    flat = np.frombuffer(splitmix_bytes(n * 16, 330 + n_devices), dtype=np.uint8)
    assert np.array_equal(hb.uid_parts_fixed_host(flat, 16, n_devices=n_devices), _want_fixed(oracle, flat, 16))
    rng = np.random.default_rng(331 + n_devices)
    m = 200_003
    lens = rng.integers(0, 600, size=m)
    off = np.zeros(m + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    data = rng.integers(0, 256, size=int(off[-1]), dtype=np.uint8)
    assert np.array_equal(hb.uid_parts_var_host(data, off, n_devices=n_devices),
                          oracle.uid_parts(oracle.hash_var(data, off)))
    assert np.array_equal(hb.uid_parts_fixed_host(flat[:48], 16, n_devices=n_devices),
                          _want_fixed(oracle, flat[:48], 16))  # fewer keys than shards


def test_host_uid_mixed_and_unaligned_buffers(hb, dev, oracle, monkeypatch):
    """Pageable keys with a page-locked parts output (the kernel stores the
    parts straight into it) and the reverse; a parts output 4 B off 8-B
    alignment in both kinds of memory; a fixed key longer than a staging slot."""
    lib = hb.load()
    n = 1_000_003
    flat = np.frombuffer(splitmix_bytes(n * 16 + 16, 340), dtype=np.uint8)[: n * 16]
    want = _want_fixed(oracle, flat, 16)
    pk = torch.from_numpy(flat.copy()).pin_memory()
    for keys_ptr in (flat.ctypes.data, pk.data_ptr()):
        pout = torch.zeros(2 * n + 2, dtype=torch.int32).pin_memory()  # 4-B steps: room for a misaligned start
        host = np.zeros(2 * n + 2, dtype=np.uint32)
        for base, arr in ((pout.data_ptr(), pout.numpy()), (host.ctypes.data, host)):
            for skew in (0, 4):
                arr[:] = 0
                rc = lib.shf_uid_parts_batch_fixed(keys_ptr, 16, n, 12345, base + skew, hb.MEM_HOST)
                assert rc == 0
                got = np.frombuffer(arr.view(np.uint8)[skew:skew + 8 * n].tobytes(), dtype=np.uint64)
                assert np.array_equal(got, want), (keys_ptr == pk.data_ptr(), base == host.ctypes.data, skew)
    monkeypatch.setenv("SHF_HB_STAGE_MB", "1")
    big = (1 << 20) + 4099  # longer than a 1-MiB slot: one key at a time through a device buffer of its own
    kb = np.frombuffer(splitmix_bytes(3 * big, 341), dtype=np.uint8)
    assert np.array_equal(hb.uid_parts_fixed_host(kb, big), _want_fixed(oracle, kb, big))


def _want_order(parts):
    w = (parts & np.uint64(0xFF)).astype(np.int64)
    perm = np.argsort(w, kind="stable").astype(np.uint32)
    ws = np.zeros(257, dtype=np.uint32)
    ws[1:] = np.cumsum(np.bincount(w, minlength=256))
    return perm, ws


@pytest.mark.parametrize("key_len", [16, 24, 256])
def test_uid_parts_win_host_fixed(hb, dev, oracle, key_len):
    """shf_uid_parts_batch_fixed_win, host memory: the parts, and the window
    order a stable sort of their window byte gives (= shf_win_order of the
    batch's hashes), with each window's first position."""
    n = 1_000_003
    flat = np.frombuffer(splitmix_bytes(n * key_len, 350 + key_len), dtype=np.uint8)
    parts, perm, ws = hb.uid_parts_fixed_win_host(flat, key_len)
    want = _want_fixed(oracle, flat, key_len)
    assert np.array_equal(parts, want)
    wp, wws = _want_order(want)
    assert np.array_equal(perm, wp) and np.array_equal(ws, wws)


def test_uid_parts_win_var_and_device(hb, dev, oracle):
    """The variable-length form from host memory, both forms on device memory,
    n = 0 (win_start all zero) and a decreasing offset (refused before any copy)."""
    rng = np.random.default_rng(360)
    m = 300_001
    lens = rng.integers(0, 600, size=m)
    off = np.zeros(m + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    data = rng.integers(0, 256, size=int(off[-1]), dtype=np.uint8)
    want = oracle.uid_parts(oracle.hash_var(data, off))
    wp, wws = _want_order(want)
    parts, perm, ws = hb.uid_parts_var_win_host(data, off)
    assert np.array_equal(parts, want) and np.array_equal(perm, wp) and np.array_equal(ws, wws)
    lib = hb.load()
    d_data = torch.from_numpy(data).to(dev)
    d_off = torch.from_numpy(off.view(np.int64)).to(dev)
    d_parts = torch.empty(m, dtype=torch.int64, device=dev)
    d_perm = torch.empty(m, dtype=torch.int32, device=dev)
    d_ws = torch.empty(257, dtype=torch.int32, device=dev)
    assert lib.shf_uid_parts_batch_var_win(d_data.data_ptr(), d_off.data_ptr(), m, 12345, d_parts.data_ptr(),
                                           d_perm.data_ptr(), d_ws.data_ptr(), hb.MEM_DEVICE) == 0
    assert np.array_equal(d_parts.cpu().numpy().view(np.uint64), want)
    assert np.array_equal(d_perm.cpu().numpy().view(np.uint32), wp)
    assert np.array_equal(d_ws.cpu().numpy().view(np.uint32), wws)
    n = 500_000
    keys = torch.randint(0, 256, (n * 16,), dtype=torch.uint8, device=dev)
    f_parts = torch.empty(n, dtype=torch.int64, device=dev)
    f_perm = torch.empty(n, dtype=torch.int32, device=dev)
    assert lib.shf_uid_parts_batch_fixed_win(keys.data_ptr(), 16, n, 12345, f_parts.data_ptr(), f_perm.data_ptr(),
                                             None, hb.MEM_DEVICE) == 0
    fwant = _want_fixed(oracle, keys.cpu().numpy(), 16)
    assert np.array_equal(f_parts.cpu().numpy().view(np.uint64), fwant)
    assert np.array_equal(f_perm.cpu().numpy().view(np.uint32), _want_order(fwant)[0])
    z = np.full(257, 7, dtype=np.uint32)
    assert lib.shf_uid_parts_batch_fixed_win(None, 16, 0, 12345, None, None, z.ctypes.data, hb.MEM_HOST) == 0
    assert not z.any()
    bad = off.copy()
    bad[10] = bad[9] - np.uint64(1)
    out = np.zeros(m, dtype=np.uint64)
    pm = np.zeros(m, dtype=np.uint32)
    assert lib.shf_uid_parts_batch_var_win(data.ctypes.data, bad.ctypes.data, m, 12345, out.ctypes.data,
                                           pm.ctypes.data, None, hb.MEM_HOST) == hb.ERR_ARG
    assert not out.any()
