"""Robustness of the product path on the GPU (through the C ABI):

* malformed device-resident offsets (include/shf_hash_batch.h Conventions): the
  kernels skip invalid keys without reading their bytes, still hash every valid
  key bit-exact, and the call reports SHF_HB_ERR_ARG (sync) or through
  shf_hash_batch_status() (async) -- never a GPU fault;
* the Python binding's argument checks (dtype, device, shape) before any launch;
* per-thread resources: short-lived caller threads leave nothing behind, and
  concurrent threads share one bounded staging pool (the reference's usage
  model is many processes and threads on one box, /root/reference/README.md:47-49);
* the multi-device split (run_multi) with several host threads sharing one GPU
  (test-only knob SHF_HB_MULTI_SHARE_DEVICES).
"""
import ctypes
import gc
import threading

import numpy as np
import pytest

from sharedhashfile_amd.keygen import splitmix_bytes

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

SENTINEL = np.uint64(0xDEADBEEFDEADBEEF)
VAR_KERNELS = [0, 3, 4, 5, 6]  # AUTO, GENERIC, SPAN, ROUND, SPAN_PP


@pytest.fixture(scope="module")
def dev(hb):
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    hb.check_device()
    return torch.device("cuda:0")


def _malformed(n=1000, seed=3):
    """A batch with invalid keys: 99 (offsets decrease), 499 (length 2^31), 500
    (it starts at 499's end: decreasing), 777 (length 2^31 + 5) and 778."""
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 300, size=n)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    data = np.frombuffer(splitmix_bytes(int(off[-1]) + 64, seed), dtype=np.uint8).copy()
    off[100] = off[99] - np.uint64(5)
    off[500] = off[499] + np.uint64(1 << 31)
    off[778] = off[777] + np.uint64((1 << 31) + 5)
    bad = {99, 499, 500, 777, 778}
    return data, off, bad


def _want(oracle, data, off, bad):
    n = off.size - 1
    want = np.empty((n, 2), dtype=np.uint64)
    for i in range(n):
        if i in bad:
            want[i] = SENTINEL
        else:
            o0, o1 = int(off[i]), int(off[i + 1])
            want[i] = oracle.hash_var(data[o0:o1], np.array([0, o1 - o0], dtype=np.uint64))[0]
    return want


def _dev_bufs(data, off, n, dev):
    d = torch.from_numpy(data).to(dev)
    o = torch.from_numpy(off.view(np.int64)).to(dev)
    out = torch.full((n, 2), int(SENTINEL.view(np.int64)), dtype=torch.int64, device=dev)
    return d, o, out


@pytest.mark.parametrize("kernel", VAR_KERNELS)
def test_malformed_offsets_async_status(hb, dev, oracle, kernel):
    lib = hb.load()
    data, off, bad = _malformed()
    n = off.size - 1
    want = _want(oracle, data, off, bad)
    d, o, out = _dev_bufs(data, off, n, dev)
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert lib.shf_hash_batch_status(s) == hb.OK  # nothing pending
    assert lib.shf_hash_batch_var_kernel_async(d.data_ptr(), o.data_ptr(), n, 12345, out.data_ptr(), kernel, s) == 0
    assert lib.shf_hash_batch_status(s) == hb.ERR_ARG
    assert lib.shf_hash_batch_status(s) == hb.OK  # the query cleared it
    assert np.array_equal(out.cpu().numpy().view(np.uint64), want)
    # sized entry point (span window from the byte count), Python binding + status()
    out.fill_(int(SENTINEL.view(np.int64)))
    hb.hash_var(d, o, out=out, kernel=kernel, key_bytes=int(off[-1]))
    with pytest.raises(hb.ShfHashBatchError) as ei:
        hb.status()
    assert ei.value.status == hb.ERR_ARG
    assert np.array_equal(out.cpu().numpy().view(np.uint64), want)


def test_malformed_offsets_sync_and_other_outputs(hb, dev, oracle):
    lib = hb.load()
    data, off, bad = _malformed(seed=4)
    n = off.size - 1
    want = _want(oracle, data, off, bad)
    d, o, out = _dev_bufs(data, off, n, dev)
    assert lib.shf_hash_batch_var(d.data_ptr(), o.data_ptr(), n, 12345, out.data_ptr(), hb.MEM_DEVICE) == hb.ERR_ARG
    assert np.array_equal(out.cpu().numpy().view(np.uint64), want)
    # a valid batch through the same sync entry point is OK again (its own status word)
    good = np.arange(0, 1001, dtype=np.uint64) * np.uint64(7)
    og = torch.from_numpy(good.view(np.int64)).to(dev)
    assert lib.shf_hash_batch_var(d.data_ptr(), og.data_ptr(), 1000, 12345, out.data_ptr(), hb.MEM_DEVICE) == hb.OK
    # UID parts and probe (async) report through the status word
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    parts = torch.zeros(n, dtype=torch.int64, device=dev)
    assert lib.shf_uid_parts_batch_var_async(d.data_ptr(), o.data_ptr(), n, 12345, parts.data_ptr(), s) == 0
    assert lib.shf_hash_batch_status(s) == hb.ERR_ARG
    ok = np.array([i for i in range(n) if i not in bad])
    assert np.array_equal(parts.cpu().numpy().view(np.uint64)[ok], oracle.uid_parts(want[ok]))
    idx = hb.RowIndex(4)
    rec = torch.zeros((n, 4), dtype=torch.int32, device=dev)
    assert lib.shf_probe_batch_var_async(idx.handle, d.data_ptr(), o.data_ptr(), n, 12345, None, rec.data_ptr(),
                                         s) == 0
    assert lib.shf_hash_batch_status(s) == hb.ERR_ARG
    assert lib.shf_probe_batch_var(idx.handle, d.data_ptr(), o.data_ptr(), n, 12345, None, rec.data_ptr(),
                                   hb.MEM_DEVICE) == hb.ERR_ARG
    idx.close()
    torch.cuda.synchronize()


def test_python_binding_rejects_bad_arguments(hb, dev):
    keys = torch.zeros(64, dtype=torch.uint8, device=dev)
    with pytest.raises(TypeError):
        hb.hash_fixed(keys.view(torch.int64), 16)  # not uint8: would count elements, not bytes
    with pytest.raises(TypeError):
        hb.hash_fixed(torch.zeros(64, dtype=torch.uint8), 16)  # host tensor
    with pytest.raises(ValueError):
        hb.hash_fixed(keys.view(8, 8).t(), 16)  # not contiguous
    with pytest.raises(ValueError):
        hb.hash_fixed(keys, 16, out=torch.zeros((3, 2), dtype=torch.int64, device=dev))  # wrong shape
    off = torch.tensor([0, 8, 16], dtype=torch.int64, device=dev)
    with pytest.raises(TypeError):
        hb.hash_var(keys, off.to(torch.int32))
    with pytest.raises(TypeError):
        hb.hash_var(keys, off.cpu())
    with pytest.raises(ValueError):
        hb.hash_var(keys, off, out=torch.zeros((3, 2), dtype=torch.int64, device=dev))
    with pytest.raises(ValueError):
        hb.hash_var(keys, off.view(3, 1))


def test_short_lived_threads_release_their_contexts(hb, dev, oracle):
    """64 threads each hash a host batch (32 MiB of keys) and exit. Staging is
    the process pool's (a bounded set of slots, include/shf_hash_batch.h), so a
    thread keeps only a stream and a few status words per device, and those go
    when it exits: neither device nor host memory grows with the threads."""
    import psutil

    lib = hb.load()
    n = 2 << 20
    keys = np.frombuffer(splitmix_bytes(n * 16, 41), dtype=np.uint8)
    idx = np.unique(np.random.default_rng(1).integers(0, n, size=20000))
    want = oracle.hash_fixed(keys.reshape(n, 16)[idx], 16)
    results = []

    def call():
        out = np.empty((n, 2), dtype=np.uint64)
        rc = lib.shf_hash_batch_fixed(keys.ctypes.data, 16, n, 12345, out.ctypes.data, hb.MEM_HOST)
        results.append(rc == 0 and np.array_equal(out[idx], want))

    def wave(k):
        ts = [threading.Thread(target=call) for _ in range(k)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()

    wave(8)  # the pool's slots and the copy workers exist from here on
    gc.collect()
    proc = psutil.Process()
    rss0, free0 = proc.memory_info().rss, torch.cuda.mem_get_info()[0]
    for _ in range(8):
        wave(8)
    gc.collect()
    rss1, free1 = proc.memory_info().rss, torch.cuda.mem_get_info()[0]
    assert len(results) == 72 and all(results)
    leaked_host, leaked_dev = rss1 - rss0, free0 - free1
    print("64 threads: device %+.1f MiB, host RSS %+.1f MiB" % (leaked_dev / 2**20, leaked_host / 2**20))
    assert leaked_dev < (512 << 20), leaked_dev
    assert leaked_host < (512 << 20), leaked_host


def test_concurrent_threads_share_the_staging_pool(hb, dev, oracle):
    """16 threads hash 10M x 16-B pageable batches at once (SharedHashFile's
    many-threads-per-box model, /root/reference/src/test.f.shf.c:274-336): the
    device memory in use while they run stays within the pool's footprint
    (SHF_HB_POOL_MB, default 64 MiB) plus a small per-thread allowance, where
    per-thread staging would take 16 x 80 MiB; every result is bit-exact."""
    lib = hb.load()
    n, threads = 10_000_000, 16
    keys = np.frombuffer(splitmix_bytes(n * 16, 71), dtype=np.uint8)
    idx = np.unique(np.random.default_rng(2).integers(0, n, size=20000))
    want = oracle.hash_fixed(keys.reshape(n, 16)[idx], 16)
    outs = [np.empty((n, 2), dtype=np.uint64) for _ in range(threads)]

    def warm(i):  # the same wave once, so that what the HIP runtime keeps for it (queues, signals) exists
        lib.shf_hash_batch_fixed(keys.ctypes.data, 16, n, 12345, outs[i].ctypes.data, hb.MEM_HOST)

    ws = [threading.Thread(target=warm, args=(i,)) for i in range(threads)]
    for t in ws:
        t.start()
    for t in ws:
        t.join()
    assert lib.shf_hash_batch_release() == 0  # the library's own state and slots freed: measured from nothing
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info()[0]
    rcs, low = [], [free0]
    stop = threading.Event()

    def sample():
        while not stop.is_set():
            low[0] = min(low[0], torch.cuda.mem_get_info()[0])
            stop.wait(0.002)

    def call(i):
        rcs.append(lib.shf_hash_batch_fixed(keys.ctypes.data, 16, n, 12345, outs[i].ctypes.data, hb.MEM_HOST))

    sampler = threading.Thread(target=sample)
    sampler.start()
    ts = [threading.Thread(target=call, args=(i,)) for i in range(threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    stop.set()
    sampler.join()
    low[0] = min(low[0], torch.cuda.mem_get_info()[0])
    assert rcs == [0] * threads
    for o in outs:
        assert np.array_equal(o[idx], want)
    peak = free0 - low[0]
    after = free0 - torch.cuda.mem_get_info()[0]
    # one thread alone, from nothing: the pool's slots it makes
    assert lib.shf_hash_batch_release() == 0
    f1 = torch.cuda.mem_get_info()[0]
    call(0)
    single = f1 - torch.cuda.mem_get_info()[0]
    msg = "peak %.1f MiB during, %.1f MiB after the 16 threads; one thread alone %.1f MiB" % (
        peak / 2**20, after / 2**20, single / 2**20)
    print(msg)
    # what the library holds: the pool's 64 MiB of slots and a stream + status words per thread
    assert after <= (64 << 20) + threads * (2 << 20), msg
    assert single <= (64 << 20) + (8 << 20), msg
    # while the calls run the HIP runtime adds buffers of its own per stream in use; per-thread
    # staging (round 4) would need 16 x 80 MiB = 1.25 GiB on top
    assert peak <= (384 << 20), msg
    # the pool keeps its slots for the next call; release frees the idle ones
    assert lib.shf_hash_batch_release() == 0
    assert torch.cuda.mem_get_info()[0] >= free0 - (8 << 20)


def test_a_parked_context_starts_clean(hb, dev, oracle):
    """A thread that exits leaves its per-device state parked for the next
    thread (no HIP call at thread exit): a status a dead thread never queried
    must not reach the thread that picks its state up, and release() frees
    every parked context (include/shf_hash_batch.h shf_hash_batch_release)."""
    lib = hb.load()
    data, off, bad = _malformed(seed=9)
    n = off.size - 1
    d, o, out = _dev_bufs(data, off, n, dev)
    torch.cuda.synchronize()
    seen = {}

    def dirty():  # an async call that flags a bad key, never queried; the thread exits
        s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        seen["dirty"] = lib.shf_hash_batch_var_async(d.data_ptr(), o.data_ptr(), n, 12345, out.data_ptr(), s)
        torch.cuda.synchronize()

    def clean():  # the next thread (likely on the parked state): nothing pending
        s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        seen["clean"] = lib.shf_hash_batch_status(s)
        keys = np.frombuffer(splitmix_bytes(70_000 * 16, 91), dtype=np.uint8)
        got = np.empty((70_000, 2), dtype=np.uint64)
        seen["host"] = lib.shf_hash_batch_fixed(keys.ctypes.data, 16, 70_000, 12345, got.ctypes.data, hb.MEM_HOST)
        seen["ok"] = np.array_equal(got, oracle.hash_fixed(keys, 16))

    for f in (dirty, clean, clean):
        t = threading.Thread(target=f)
        t.start()
        t.join()
    assert seen["dirty"] == 0 and seen["clean"] == hb.OK and seen["host"] == 0 and seen["ok"]
    assert lib.shf_hash_batch_release() == 0
    # and everything starts afresh afterwards, on this thread and on a new one
    assert lib.shf_hash_batch_status(ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)) == hb.OK
    t = threading.Thread(target=clean)
    t.start()
    t.join()
    assert seen["clean"] == hb.OK and seen["ok"]


@pytest.mark.parametrize("pool_mb", ["1", "32"])
def test_threads_wait_for_slots_of_a_small_pool(hb, dev, oracle, monkeypatch, pool_mb):
    """8 threads, fixed- and variable-length host batches at once, through a
    pool of one slot (1 MiB: less than one 16-MiB slot still makes one) or two:
    a call waits only for its first slot, none waits while holding one, and
    every result is bit-exact."""
    monkeypatch.setenv("SHF_HB_POOL_MB", pool_mb)
    lib = hb.load()
    n = 1_500_007
    keys = np.frombuffer(splitmix_bytes(n * 16, 81), dtype=np.uint8)
    want = oracle.hash_fixed(keys, 16, threads=8)
    rng = np.random.default_rng(82)
    m = 150_001
    lens = rng.integers(0, 600, size=m)
    off = np.zeros(m + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    data = rng.integers(0, 256, size=int(off[-1]), dtype=np.uint8)
    vwant = oracle.hash_var(data, off)
    ok = []

    def call(i):
        if i % 2:
            out = np.empty((n, 2), dtype=np.uint64)
            rc = lib.shf_hash_batch_fixed(keys.ctypes.data, 16, n, 12345, out.ctypes.data, hb.MEM_HOST)
            ok.append(rc == 0 and np.array_equal(out, want))
        else:
            out = np.empty((m, 2), dtype=np.uint64)
            rc = lib.shf_hash_batch_var(data.ctypes.data, off.ctypes.data, m, 12345, out.ctypes.data, hb.MEM_HOST)
            ok.append(rc == 0 and np.array_equal(out, vwant))

    ts = [threading.Thread(target=call, args=(i,)) for i in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in ts), "a call never got a slot"
    assert ok == [True] * 8


def test_processes_hash_at_once(hb, dev, oracle, tmp_path):
    """The reference's multi-process model (test.f.shf.c:274-336: children that
    each put their own key range): four processes, each with its own staging
    pool and contexts, hash their ranges of one batch through the host and the
    device paths at the same time; every result bit-exact."""
    import subprocess
    import sys

    n, procs = 400_000, 4
    keys = np.frombuffer(splitmix_bytes(n * 16, 95), dtype=np.uint8).copy()
    src = tmp_path / "keys.bin"
    keys.tofile(src)
    child = r"""
import sys, numpy as np, torch
sys.path.insert(0, sys.argv[4])
import sharedhashfile_amd as hb
lo, hi = int(sys.argv[2]), int(sys.argv[3])
keys = np.fromfile(sys.argv[1], dtype=np.uint8)[lo * 16:hi * 16].copy()
out = np.empty((hi - lo, 2), dtype=np.uint64)
assert hb.load().shf_hash_batch_fixed(keys.ctypes.data, 16, hi - lo, 12345, out.ctypes.data, hb.MEM_HOST) == 0
d = hb.hash_fixed(torch.from_numpy(keys).to("cuda:0"), 16)
torch.cuda.synchronize()
assert np.array_equal(d.cpu().numpy().view(np.uint64), out)
out.tofile(sys.argv[1] + ".%d" % lo)
"""
    root = str(__import__("pathlib").Path(__file__).resolve().parents[1])
    ps = [subprocess.Popen([sys.executable, "-c", child, str(src), str(n * i // procs), str(n * (i + 1) // procs), root],
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for i in range(procs)]
    for p in ps:
        _, err = p.communicate(timeout=180)
        assert p.returncode == 0, err[-2000:]
    want = oracle.hash_fixed(keys, 16, threads=8)
    got = np.concatenate([np.fromfile(str(src) + ".%d" % (n * i // procs), dtype=np.uint64).reshape(-1, 2)
                          for i in range(procs)])
    assert np.array_equal(got, want)


@pytest.mark.parametrize("n_devices", [2, 3])
def test_multi_split_with_shared_device(hb, dev, oracle, monkeypatch, n_devices):
    """shf_hash_batch_*_multi's split (one host thread per shard, contiguous key
    ranges, results into disjoint slices) with the shards sharing this GPU."""
    monkeypatch.setenv("SHF_HB_MULTI_SHARE_DEVICES", "1")
    n = 1_000_003
    flat = np.frombuffer(splitmix_bytes(n * 16, 51), dtype=np.uint8)
    assert np.array_equal(hb.hash_fixed_host(flat, 16, n_devices=n_devices), oracle.hash_fixed(flat, 16, threads=8))
    rng = np.random.default_rng(n_devices)
    m = 200_001
    lens = rng.integers(0, 600, size=m)
    off = np.zeros(m + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    data = rng.integers(0, 256, size=int(off[-1]), dtype=np.uint8)
    assert np.array_equal(hb.hash_var_host(data, off, n_devices=n_devices), oracle.hash_var(data, off))
    # fewer keys than shards: the split shrinks, nothing is dropped
    assert np.array_equal(hb.hash_fixed_host(flat[:32], 16, n_devices=n_devices), oracle.hash_fixed(flat[:32], 16))


def test_host_keys_larger_than_the_stage(hb, dev, oracle, monkeypatch):
    """A fixed key and a variable key larger than SHF_HB_STAGE_MB go through a
    temporary device buffer (the slots keep their stage size)."""
    monkeypatch.setenv("SHF_HB_STAGE_MB", "1")
    big = (1 << 20) + 4099
    flat = np.frombuffer(splitmix_bytes(3 * big, 61), dtype=np.uint8)
    assert np.array_equal(hb.hash_fixed_host(flat, big), oracle.hash_fixed(flat, big))
    off = np.array([0, 10, 10 + 3 * big - 100, 3 * big - 50, 3 * big], dtype=np.uint64)
    assert np.array_equal(hb.hash_var_host(flat, off), oracle.hash_var(flat, off))


def test_eight_shards_share_the_copy_workers(hb, dev, oracle, monkeypatch):
    """What an 8-GPU host caller hits: shf_hash_batch_*_multi
    with n_devices = 8 from pageable buffers -- 8 shard threads whose chunks'
    copy-outs (drain_async pieces that wait on each slot's event) share the one
    pool of <= 12 copy workers with the staging copies -- here on one GPU
    (SHF_HB_MULTI_SHARE_DEVICES). configs[4]'s 16-B keys at 100M and configs[3]'s
    U[8,512] B at 10M: every key against the device kernels, a sample against
    the oracle, and each call within a stated wall time (10 s; an unshared run
    takes well under 1 s, so only a stall of the shared workers reaches it)."""
    import time

    from sharedhashfile_amd.keygen import device_random_bytes

    monkeypatch.setenv("SHF_HB_MULTI_SHARE_DEVICES", "1")
    limit_s = 10.0
    n = 100_000_000
    keys = device_random_bytes(n * 16, 401, dev)
    ref = hb.hash_fixed(keys, 16)
    host = keys.cpu().numpy()
    del keys
    times = []
    for _ in range(2):  # the second call finds the workers and slots made
        t0 = time.perf_counter()
        got = hb.hash_fixed_host(host, 16, n_devices=8)
        times.append(time.perf_counter() - t0)
    assert torch.equal(torch.from_numpy(got.view(np.int64)).to(dev), ref)
    del ref
    idx = np.unique(np.concatenate([np.random.default_rng(401).integers(0, n, size=20000), [0, n - 1]]))
    assert np.array_equal(got[idx], oracle.hash_fixed(host.reshape(n, 16)[idx], 16))
    del got, host
    m = 10_000_000
    g = torch.Generator(device=dev)
    g.manual_seed(402)
    lens = torch.randint(8, 513, (m,), generator=g, device=dev, dtype=torch.int64)
    off = torch.zeros(m + 1, dtype=torch.int64, device=dev)
    torch.cumsum(lens, 0, out=off[1:])
    del lens
    data = device_random_bytes(int(off[-1].item()), 403, dev)
    vref = hb.hash_var(data, off)
    h_data, h_off = data.cpu().numpy(), off.cpu().numpy().view(np.uint64)
    del data, off
    vtimes = []
    for _ in range(2):
        t0 = time.perf_counter()
        vgot = hb.hash_var_host(h_data, h_off, n_devices=8)
        vtimes.append(time.perf_counter() - t0)
    assert torch.equal(torch.from_numpy(vgot.view(np.int64)).to(dev), vref)
    vidx = np.unique(np.random.default_rng(402).integers(0, m, size=2000))
    sub_off = np.zeros(len(vidx) + 1, dtype=np.uint64)
    sub_off[1:] = np.cumsum(h_off[vidx + 1] - h_off[vidx])
    sub = np.concatenate([h_data[h_off[i]:h_off[i + 1]] for i in vidx])
    assert np.array_equal(vgot[vidx], oracle.hash_var(sub, sub_off))
    print("8 shards on one GPU: 100M x 16 B %s s (%.2f G keys/s), 10M x U[8,512] B %s s (%.3f G keys/s)" % (
        ["%.3f" % t for t in times], n / min(times) / 1e9, ["%.3f" % t for t in vtimes], m / min(vtimes) / 1e9))
    assert max(times) < limit_s and max(vtimes) < limit_s, (times, vtimes)
