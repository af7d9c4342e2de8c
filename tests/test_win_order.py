"""Window order of a batch (shf_win_order*, csrc/win_order.hip).

perm = the key indices stably sorted by win = h1 & 0xff, the window the
reference's put/get/del take from the hash (/root/reference/src/shf.c:800,
:893). The claim that makes the order useful is that it changes nothing: every
structure an operation touches belongs to its key's window (lock, tab2 -> tab
map, tabs numbered per window, shf.c:432), so a batch replayed window by
window, batch order kept inside each window, leaves the reference's store byte
for byte as batch order does, with the same uids. That claim is checked here
against the reference's own put/get (oracle/_ref/libref_shf.so): on the CPU
with the oracle's order, and on the GPU with the library's hashes and order.
The order itself is checked bit-exact against the numpy restatement
(Oracle.win_order: a stable argsort).
"""
import os
import tempfile

import numpy as np
import pytest

from oracle.oracle_py import REF_SO, Oracle, reference_put_in_order, store_files

SHM = "/dev/shm" if os.path.isdir("/dev/shm") else None


def _unique_keys(n, seed, lo=4, hi=120):
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


def _same_store(data, off, hashes, perm, lockable=1):
    """Puts the batch in batch order and in perm order into two fresh reference
    stores; returns both results after checking the stores are identical."""
    with tempfile.TemporaryDirectory(dir=SHM) as d:
        a = reference_put_in_order(data, off, hashes, None, d, "batch", lockable)
        b = reference_put_in_order(data, off, hashes, perm, d, "winord", lockable)
        fa = store_files(d, "batch")
        fb = {k.replace("winord", "batch"): v for k, v in store_files(d, "winord").items()}
    n = off.size - 1
    assert a[0] == n and b[0] == n  # every key found with its value, in either order
    np.testing.assert_array_equal(a[1], b[1])  # the same uid for every key
    assert sorted(fa) == sorted(fb) and len(fa) == 257  # 256 window folders' files + the store file
    assert [k for k in fa if fa[k] != fb[k]] == []  # byte for byte
    return a, b


def test_oracle_order_is_a_stable_window_sort(oracle):
    rng = np.random.default_rng(3)
    h = rng.integers(0, 2**63, size=(5000, 2), dtype=np.int64).astype(np.uint64)
    h[::7, 0] = (h[::7, 0] & ~np.uint64(0xFF)) | np.uint64(17)  # a crowded window
    perm, start = Oracle.win_order(h)
    assert sorted(perm.tolist()) == list(range(5000))
    w = (h[perm, 0] & np.uint64(0xFF)).astype(np.int64)
    assert (np.diff(w) >= 0).all()
    for win in (17, int(w[0]), int(w[-1])):
        run = perm[start[win]:start[win + 1]]
        assert (w[start[win]:start[win + 1]] == win).all() and (np.diff(run.astype(np.int64)) > 0).all()
    assert start[0] == 0 and start[256] == 5000


@pytest.mark.skipif(not os.path.exists(REF_SO), reason="oracle/_ref/libref_shf.so not built")
@pytest.mark.parametrize("lockable", [1, 0])
def test_window_order_leaves_the_reference_store_identical(oracle, lockable):
    """The reference's own put/get over 60 000 keys (enough that tabs part,
    shf.c:829-834) in batch order and in window order: identical files, uids
    and values."""
    data, off = _unique_keys(60000, 11)
    h = oracle.hash_var(data, off)
    perm, _ = Oracle.win_order(h)
    _same_store(data, off, h, perm, lockable)


# ---------------------------------------------------------------------------
# GPU: the library's order against the oracle, and end to end
# ---------------------------------------------------------------------------
@pytest.fixture(scope="module")
def dev(hb):
    import torch

    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    hb.check_device()  # raises unless the current device is gfx950
    return torch.device("cuda:0")


def _rand_hashes(n, seed, wins=None):
    rng = np.random.default_rng(seed)
    h = rng.integers(0, 2**63, size=(n, 2), dtype=np.int64).astype(np.uint64)
    if wins is not None:
        h[:, 0] = (h[:, 0] & ~np.uint64(0xFF)) | np.asarray(wins, dtype=np.uint64)
    return h


def _gpu_order(hb, dev, h, **kw):
    import torch

    t = torch.from_numpy(h.view(np.int64)).to(dev)
    perm, start = hb.win_order(t, **kw)
    torch.cuda.synchronize(dev)
    return perm.cpu().numpy().view(np.uint32), start.cpu().numpy().view(np.uint32)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 1, 63, 64, 65, 4095, 4096, 4097, 4 * 4096 + 1, 64 * 4096, 64 * 4096 + 1, 100_003,
                               1_234_567, 10_000_003])
def test_win_order_matches_oracle(hb, dev, n):
    h = _rand_hashes(n, n)
    perm, start = _gpu_order(hb, dev, h)
    ref_perm, ref_start = Oracle.win_order(h)
    np.testing.assert_array_equal(perm, ref_perm)
    np.testing.assert_array_equal(start, ref_start)


@pytest.mark.gpu
@pytest.mark.parametrize("pattern", ["one", "two", "descending", "runs", "zero_and_255"])
def test_win_order_skewed_windows(hb, dev, pattern):
    """Every key in one window (every step's 64 lanes peers), two windows,
    windows descending, long runs, only windows 0 and 255 (all eight ballots
    agree / disagree)."""
    n = 3 * 4096 + 77
    i = np.arange(n)
    wins = {"one": np.full(n, 200), "two": (i % 2) * 255, "descending": 255 - (i * 256 // n),
            "runs": (i // 1000) % 256, "zero_and_255": np.where(i % 3 == 0, 0, 255)}[pattern]
    h = _rand_hashes(n, 5, wins)
    perm, start = _gpu_order(hb, dev, h)
    ref_perm, ref_start = Oracle.win_order(h)
    np.testing.assert_array_equal(perm, ref_perm)
    np.testing.assert_array_equal(start, ref_start)


@pytest.mark.gpu
def test_win_order_of_library_hashes_side_stream_and_host(hb, dev, oracle):
    """Hashes made by the library, the order enqueued on a side stream with a
    caller workspace; the synchronous host-memory entry point agrees."""
    import torch

    data, off = _unique_keys(200_000, 2, 1, 300)
    ref_h = oracle.hash_var(data, off)
    d = torch.from_numpy(data).to(dev)
    o = torch.from_numpy(off.view(np.int64)).to(dev)
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        h = hb.hash_var(d, o, stream=s)
        ws = torch.empty(hb.load().shf_win_order_workspace_bytes(h.shape[0]), dtype=torch.uint8, device=dev)
        perm, start = hb.win_order(h, workspace=ws, stream=s)
    s.synchronize()
    np.testing.assert_array_equal(h.cpu().numpy().view(np.uint64), ref_h)
    ref_perm, ref_start = Oracle.win_order(ref_h)
    np.testing.assert_array_equal(perm.cpu().numpy().view(np.uint32), ref_perm)
    np.testing.assert_array_equal(start.cpu().numpy().view(np.uint32), ref_start)
    hp, hs = hb.win_order_host(ref_h)
    np.testing.assert_array_equal(hp, ref_perm)
    np.testing.assert_array_equal(hs, ref_start)
    hp0, hs0 = hb.win_order_host(np.zeros((0, 2), dtype=np.uint64))
    assert hp0.size == 0 and (hs0 == 0).all()


@pytest.mark.gpu
def test_win_order_rejects_bad_arguments(hb, dev):
    import ctypes

    import torch

    lib = hb.load()
    h = torch.zeros((10000, 2), dtype=torch.int64, device=dev)
    p = torch.empty(10000, dtype=torch.int32, device=dev)
    need = lib.shf_win_order_workspace_bytes(10000)
    ws = torch.empty(need, dtype=torch.uint8, device=dev)
    vp = lambda t: ctypes.c_void_p(t.data_ptr())
    with torch.cuda.device(dev):
        assert lib.shf_win_order_async(vp(h), 10000, vp(p), None, vp(ws), need - 1, None) == hb.ERR_ARG
        assert lib.shf_win_order_async(vp(h), 10000, None, None, vp(ws), need, None) == hb.ERR_ARG
        assert lib.shf_win_order_async(vp(h), 1 << 32, vp(p), None, vp(ws), need, None) == hb.ERR_ARG
        assert lib.shf_win_order(vp(h), 10000, vp(p), None, 7) == hb.ERR_ARG
        ws2 = torch.empty(need + 16, dtype=torch.uint8, device=dev)
        assert lib.shf_win_order_async(vp(h), 10000, vp(p), None, ctypes.c_void_p(ws2.data_ptr() + 4), need, None) \
            == hb.ERR_ARG  # a workspace slice off 16-B alignment
        assert lib.shf_win_order_async(vp(h), 10000, vp(p), None, vp(ws), need, None) == hb.OK
    torch.cuda.synchronize(dev)


@pytest.mark.gpu
def test_win_order_on_a_side_stream_outside_its_context(hb, dev, oracle):
    """stream= given without `with torch.cuda.stream(s)`: the wrapper's own
    workspace stays reserved for that stream until its kernels ran,
    so churning the allocator on the current stream meanwhile cannot corrupt it."""
    import torch

    rng = np.random.default_rng(31)
    hn = rng.integers(0, 2**63, size=(300_000, 2), dtype=np.int64)
    h = torch.from_numpy(hn).to(dev)
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    want_p, want_s = oracle.win_order(hn.view(np.uint64))
    for _ in range(3):
        perm, ws = hb.win_order(h, stream=s)
        junk = [torch.full((1 << 20,), 7, dtype=torch.uint8, device=dev) for _ in range(8)]  # reuse freed blocks
        del junk
        s.synchronize()
        np.testing.assert_array_equal(perm.cpu().numpy().view(np.uint32), want_p)
        np.testing.assert_array_equal(ws.cpu().numpy().view(np.uint32), want_s)


@pytest.mark.gpu
def test_fused_outputs_on_a_side_stream_outside_its_context(hb, dev, oracle):
    """The same for the fused calls and the plain hash: every tensor the wrapper
    allocates (records, perm, win_start, workspace) is reserved for the stream
    the kernels run on, so allocator churn on the current stream meanwhile
    cannot overwrite them before those kernels ran."""
    import torch

    rng = np.random.default_rng(37)
    n = 200_000
    kn = rng.integers(0, 256, size=n * 16, dtype=np.uint8)
    keys = torch.from_numpy(kn).to(dev)
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    want_h = oracle.hash_fixed(kn, 16)
    want_p, want_s = oracle.win_order(want_h)
    for _ in range(3):
        h, perm, start = hb.hash_fixed_win(keys, 16, stream=s)
        h2 = hb.hash_fixed(keys, 16, stream=s)
        junk = [torch.full((1 << 20,), 7, dtype=torch.uint8, device=dev) for _ in range(16)]  # reuse freed blocks
        del junk
        s.synchronize()
        np.testing.assert_array_equal(h.cpu().numpy().view(np.uint64), want_h)
        np.testing.assert_array_equal(h2.cpu().numpy().view(np.uint64), want_h)
        np.testing.assert_array_equal(perm.cpu().numpy().view(np.uint32), want_p)
        np.testing.assert_array_equal(start.cpu().numpy().view(np.uint32), want_s)


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(REF_SO), reason="oracle/_ref/libref_shf.so not built")
def test_gpu_window_order_drives_the_reference_put(hb, dev, oracle):
    """End to end: GPU hashes and GPU window order drive the reference's own
    put and get (60 000 keys); the store equals the batch-order store byte for
    byte. The loops' times are printed (the order's point: the reference's get
    finds its window in cache)."""
    data, off = _unique_keys(60000, 12)
    h = hb.hash_var_host(data, off)
    np.testing.assert_array_equal(h, oracle.hash_var(data, off))
    perm, _ = hb.win_order_host(h)
    a, b = _same_store(data, off, h, perm)
    print("put batch order %.0f ns/key, window order %.0f; get %.0f vs %.0f ns/key"
          % (a[2] / 60000 * 1e9, b[2] / 60000 * 1e9, a[3] / 60000 * 1e9, b[3] / 60000 * 1e9))


@pytest.mark.skipif(not os.path.exists(REF_SO), reason="oracle/_ref/libref_shf.so not built")
def test_window_disjoint_workers_put_and_find_every_key(oracle):
    """What win_start is for: 4 forked worker processes of the reference (each
    its own handle, the reference's multi-process use) take whole windows of
    the window order, and every key is put and found with its value; the same
    with batch-order ranges. (CPU only: the workers are forked, and a -m gpu
    run's process has touched the GPU.)"""
    from oracle.oracle_py import reference_put_get_procs

    data, off = _unique_keys(80000, 21)
    h = oracle.hash_var(data, off)
    perm, start = Oracle.win_order(h)
    n = off.size - 1
    for order, starts in ((None, [0, n // 4, n // 2, 3 * n // 4, n]),
                          (perm, [start[0], start[64], start[128], start[192], start[256]])):
        with tempfile.TemporaryDirectory(dir=SHM) as d:
            found, _, _ = reference_put_get_procs(data, off, h, order, np.array(starts, np.uint64), d, "w", 1)
        assert found == n


# ---------------------------------------------------------------------------
# hash + window order in one call (shf_hash_batch_*_win_async): the records
# bit-exact against the oracle, the order exactly the oracle's order of them
# ---------------------------------------------------------------------------
def _check_fused(out, perm, start, want_h):
    import torch

    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint64), want_h)
    ref_perm, ref_start = Oracle.win_order(want_h)
    np.testing.assert_array_equal(perm.cpu().numpy().view(np.uint32), ref_perm)
    np.testing.assert_array_equal(start.cpu().numpy().view(np.uint32), ref_start)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 63, 4095, 4096, 4097, 3 * 4096 + 77, 100_003, 1_000_001])
@pytest.mark.parametrize("kernel", ["auto", "fixed16", "generic"])
def test_fused_fixed16_hash_and_order(hb, dev, oracle, n, kernel):
    """16-B keys: AUTO and FIXED16 run the fused kernel (k_fixed16_win: records,
    window bytes and chunk histograms in one pass); GENERIC the per-key epilogue
    (window bytes only, the chunks counted after)."""
    import torch

    rng = np.random.default_rng(n)
    keys = rng.integers(0, 256, size=n * 16, dtype=np.uint8)
    k = {"auto": hb.KERNEL_AUTO, "fixed16": hb.KERNEL_FIXED16, "generic": hb.KERNEL_GENERIC}[kernel]
    out, perm, start = hb.hash_fixed_win(torch.from_numpy(keys).to(dev), 16, kernel=k)
    _check_fused(out, perm, start, oracle.hash_fixed(keys, 16))


@pytest.mark.gpu
@pytest.mark.parametrize("key_len,kernel", [(256, "auto"), (256, "tiled"), (37, "auto"), (100, "span"), (8, "auto")])
def test_fused_fixed_other_lengths(hb, dev, oracle, key_len, kernel):
    import torch

    n = 2 * 4096 + 321
    rng = np.random.default_rng(key_len)
    keys = rng.integers(0, 256, size=n * key_len, dtype=np.uint8)
    k = {"auto": hb.KERNEL_AUTO, "tiled": hb.KERNEL_TILED, "span": hb.KERNEL_SPAN}[kernel]
    out, perm, start = hb.hash_fixed_win(torch.from_numpy(keys).to(dev), key_len, kernel=k)
    _check_fused(out, perm, start, oracle.hash_fixed(keys, key_len))


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", ["auto", "span", "span_pp", "round", "generic"])
def test_fused_var_hash_and_order(hb, dev, oracle, kernel):
    import torch

    data, off = _unique_keys(50_000, 21, 0, 512)
    k = {"auto": hb.KERNEL_AUTO, "span": hb.KERNEL_SPAN, "span_pp": hb.KERNEL_SPAN_PP, "round": hb.KERNEL_ROUND,
         "generic": hb.KERNEL_GENERIC}[kernel]
    out, perm, start = hb.hash_var_win(torch.from_numpy(data).to(dev), torch.from_numpy(off.view(np.int64)).to(dev),
                                       kernel=k)
    _check_fused(out, perm, start, oracle.hash_var(data, off))


@pytest.mark.gpu
def test_fused_order_at_config_b_size(hb, dev, oracle):
    """10M x 16-B keys (BASELINE configs[1]): the fused order equals the order of
    the library's own records (size-independent property), sampled records
    bit-exact against the oracle."""
    import torch

    from sharedhashfile_amd.keygen import device_random_bytes

    n = 10_000_000
    keys = device_random_bytes(n * 16, 77, dev)
    out, perm, start = hb.hash_fixed_win(keys, 16)
    p2, s2 = hb.win_order(out)
    torch.cuda.synchronize()
    assert torch.equal(perm, p2) and torch.equal(start, s2)
    idx = np.random.default_rng(1).integers(0, n, size=20000)
    ti = torch.from_numpy(idx).to(dev)
    got = out.index_select(0, ti).cpu().numpy().view(np.uint64)
    np.testing.assert_array_equal(got, oracle.hash_fixed(keys.view(n, 16).index_select(0, ti).cpu().numpy(), 16))
    w = (out[:, 0] & 0xFF).to(torch.int64)
    assert torch.equal(torch.bincount(w, minlength=256).cpu(), (s2[1:] - s2[:-1]).to(torch.int64).cpu())


@pytest.mark.gpu
def test_fused_rejects_bad_arguments(hb, dev):
    import ctypes

    import torch

    lib = hb.load()
    n = 5000
    keys = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    out = torch.empty((n, 2), dtype=torch.int64, device=dev)
    p = torch.empty(n, dtype=torch.int32, device=dev)
    need = lib.shf_win_order_workspace_bytes(n)
    ws = torch.empty(need + 16, dtype=torch.uint8, device=dev)
    vp = lambda t, d=0: ctypes.c_void_p(t.data_ptr() + d)
    with torch.cuda.device(dev):
        f = lib.shf_hash_batch_fixed_win_async
        assert f(vp(keys), 16, n, 12345, vp(out), vp(p), None, vp(ws), need - 1, None) == hb.ERR_ARG
        assert f(vp(keys), 16, n, 12345, vp(out), vp(p), None, vp(ws, 8), need, None) == hb.ERR_ARG
        assert f(vp(keys), 16, n, 12345, None, vp(p), None, vp(ws), need, None) == hb.ERR_ARG
        assert f(vp(keys), 16, 1 << 32, 12345, vp(out), vp(p), None, vp(ws), need, None) == hb.ERR_ARG
        assert lib.shf_hash_batch_fixed_win_kernel_async(vp(keys), 16, n, 12345, vp(out), vp(p), None, vp(ws), need,
                                                         hb.KERNEL_TILED, None) == hb.ERR_ARG
        assert lib.shf_hash_batch_var_win_kernel_async(vp(keys), vp(keys), n, 12345, vp(out), vp(p), None, vp(ws),
                                                       need, hb.KERNEL_TILED, None) == hb.ERR_ARG
        s = torch.zeros(257, dtype=torch.int32, device=dev) + 5
        assert f(None, 16, 0, 12345, None, None, vp(s), None, 0, None) == hb.OK  # empty batch: zeros
        assert f(vp(keys), 16, n, 12345, vp(out), vp(p), None, vp(ws), need, None) == hb.OK
    torch.cuda.synchronize(dev)
    assert (s == 0).all()


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 4097, 70_000, 2_500_003])
def test_fused_sync_host_fixed(hb, dev, oracle, n):
    """shf_hash_batch_fixed_win(SHF_HASH_MEM_HOST) over pageable, page-locked and
    odd-sized batches (the zero-copy, pageable zero-copy and staged pipelines all
    write the window bytes into the device workspace)."""
    import torch

    rng = np.random.default_rng(n + 5)
    keys = rng.integers(0, 256, size=n * 16, dtype=np.uint8)
    want = oracle.hash_fixed(keys, 16)
    ref_perm, ref_start = Oracle.win_order(want)
    for src in (keys, torch.from_numpy(keys.copy()).pin_memory().numpy()):
        h, perm, start = hb.hash_fixed_win_host(src.reshape(n, 16))
        np.testing.assert_array_equal(h, want)
        np.testing.assert_array_equal(perm, ref_perm)
        np.testing.assert_array_equal(start, ref_start)
    m = keys.size // 37  # the same bytes as 37-B keys (generic kernel, byte-store epilogue)
    if m:
        flat = keys[: m * 37]
        h, perm, start = hb.hash_fixed_win_host(flat.reshape(m, 37))
        np.testing.assert_array_equal(h, oracle.hash_fixed(flat, 37))
        np.testing.assert_array_equal(perm, Oracle.win_order(h)[0])


@pytest.mark.gpu
def test_fused_sync_host_var_and_device(hb, dev, oracle):
    import ctypes

    import torch

    data, off = _unique_keys(300_000, 23, 0, 600)
    want = oracle.hash_var(data, off)
    ref_perm, ref_start = Oracle.win_order(want)
    h, perm, start = hb.hash_var_win_host(data, off)
    np.testing.assert_array_equal(h, want)
    np.testing.assert_array_equal(perm, ref_perm)
    np.testing.assert_array_equal(start, ref_start)
    # device memory, synchronous
    n = off.size - 1
    d = torch.from_numpy(data).to(dev)
    o = torch.from_numpy(off.view(np.int64)).to(dev)
    out = torch.empty((n, 2), dtype=torch.int64, device=dev)
    p = torch.empty(n, dtype=torch.int32, device=dev)
    s = torch.empty(257, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    vp = lambda t: ctypes.c_void_p(t.data_ptr())
    with torch.cuda.device(dev):
        assert hb.load().shf_hash_batch_var_win(vp(d), vp(o), n, 12345, vp(out), vp(p), vp(s), hb.MEM_DEVICE) == 0
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint64), want)
    np.testing.assert_array_equal(p.cpu().numpy().view(np.uint32), ref_perm)
    np.testing.assert_array_equal(s.cpu().numpy().view(np.uint32), ref_start)
    # a decreasing offset: refused before anything moves (host), flagged by the kernels (device)
    bad = off.copy()
    bad[10] = bad[12]
    with pytest.raises(hb.ShfHashBatchError):
        hb.hash_var_win_host(data, bad)
    ob = torch.from_numpy(bad.view(np.int64)).to(dev)
    with torch.cuda.device(dev):
        assert hb.load().shf_hash_batch_var_win(vp(d), vp(ob), n, 12345, vp(out), vp(p), None, hb.MEM_DEVICE) \
            == hb.ERR_ARG
        assert hb.load().shf_hash_batch_fixed_win(vp(d), 16, 100, 12345, vp(out), vp(p), None, 9) == hb.ERR_ARG


@pytest.mark.gpu
def test_host_order_after_workspace_growth(hb, dev, oracle):
    """The synchronous host-memory order keeps its device perm buffer across a
    growth of the window-order workspace (the growth once freed the
    perm buffer too, leaving a dangling pointer that the next smaller host call
    wrote through). Host order of n1 keys, then a larger shf_win_order (grows the
    workspace), then host orders of smaller and larger batches."""
    rng = np.random.default_rng(77)
    for n, grow in ((50_000, 400_000), (20_000, 1_600_000), (30_000, 0), (900_000, 0)):
        keys = rng.integers(0, 256, size=n * 16, dtype=np.uint8)
        want = oracle.hash_fixed(keys, 16)
        h, perm, start = hb.hash_fixed_win_host(keys.reshape(n, 16))
        np.testing.assert_array_equal(h, want)
        ref_perm, ref_start = Oracle.win_order(want)
        np.testing.assert_array_equal(perm, ref_perm)
        np.testing.assert_array_equal(start, ref_start)
        if grow:
            g = _rand_hashes(grow, grow)
            gp, gs = hb.win_order_host(g)
            np.testing.assert_array_equal(gp, Oracle.win_order(g)[0])


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["fixed", "var", "fixed_win", "var_win"])
def test_sync_device_calls_follow_the_default_stream(hb, dev, oracle, kind):
    """Synchronous device-memory entry points run after the caller's work on the
    null (torch default) stream: the keys are produced there by a long chain of
    kernels and the call is made with no synchronize in between."""
    import ctypes

    import torch

    n, L = 2_000_000, 16
    vp = lambda t: ctypes.c_void_p(t.data_ptr())
    lib = hb.load()
    with torch.cuda.device(dev):
        assert torch.cuda.current_stream(dev).cuda_stream == 0
        base = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device=dev)
        keys = torch.zeros_like(base)
        torch.cuda.synchronize(dev)
        want = oracle.hash_fixed(base.cpu().numpy(), L)
        for _ in range(20):  # keep the default stream busy well past the call's launch
            keys.copy_(base)
            keys.add_(1)
            keys.sub_(1)
        out = torch.empty((n, 2), dtype=torch.int64, device=dev)
        off = torch.arange(0, (n + 1) * L, L, dtype=torch.int64, device=dev)
        perm = torch.empty(n, dtype=torch.int32, device=dev)
        start = torch.empty(257, dtype=torch.int32, device=dev)
        if kind == "fixed":
            rc = lib.shf_hash_batch_fixed(vp(keys), L, n, 12345, vp(out), hb.MEM_DEVICE)
        elif kind == "var":
            rc = lib.shf_hash_batch_var(vp(keys), vp(off), n, 12345, vp(out), hb.MEM_DEVICE)
        elif kind == "fixed_win":
            rc = lib.shf_hash_batch_fixed_win(vp(keys), L, n, 12345, vp(out), vp(perm), vp(start), hb.MEM_DEVICE)
        else:
            rc = lib.shf_hash_batch_var_win(vp(keys), vp(off), n, 12345, vp(out), vp(perm), vp(start), hb.MEM_DEVICE)
    assert rc == 0
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint64), want)
    if kind.endswith("_win"):
        ref_perm, ref_start = Oracle.win_order(want)
        np.testing.assert_array_equal(perm.cpu().numpy().view(np.uint32), ref_perm)
        np.testing.assert_array_equal(start.cpu().numpy().view(np.uint32), ref_start)
