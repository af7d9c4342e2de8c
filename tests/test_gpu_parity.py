"""Parity of the HIP path (through the C ABI) with the oracle and the reference goldens.

Bar: bit-exact, all 128 bits of every SHF_HASH (and every packed UID-parts word).
Runs only on a real MI355X: python -m pytest tests -m gpu
"""
import hashlib

import numpy as np
import pytest

from sharedhashfile_amd.keygen import counter_keys, splitmix_bytes

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev(hb):
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    hb.check_device()  # raises unless the current device is gfx950
    return torch.device("cuda:0")


def u64(t):
    torch.cuda.synchronize()
    return t.cpu().numpy().view(np.uint64)


def d_u8(a, dev):
    a = np.ascontiguousarray(a, dtype=np.uint8).reshape(-1)
    return torch.from_numpy(a if a.flags.writeable else a.copy()).to(dev)


def d_off(off, dev):
    off = np.ascontiguousarray(off, dtype=np.uint64).view(np.int64)
    return torch.from_numpy(off if off.flags.writeable else off.copy()).to(dev)


def fixed_kernels(key_len, aligned=True):
    ks = [0, 3]  # AUTO, GENERIC
    if key_len == 16 and aligned:
        ks.append(1)
    if key_len >= 32 and key_len % 16 == 0 and aligned:
        ks.append(2)
    if key_len * 64 + 16 <= 20416:
        ks.append(4)  # SPAN
    return ks


VAR_KERNELS = [0, 3, 4, 5, 6]  # AUTO, GENERIC, SPAN, ROUND, SPAN_PP


# ---------------------------------------------------------------------------
# reference goldens
# ---------------------------------------------------------------------------
def test_golden_cases(hb, dev, golden):
    for c in golden["cases"]:
        key = bytes.fromhex(c["key_hex"])
        want = np.array([int(c["h1"], 16), int(c["h2"], 16)], dtype=np.uint64)
        L = len(key)
        keys = d_u8(np.frombuffer(key, dtype=np.uint8) if L else np.zeros(16, np.uint8), dev)
        for k in fixed_kernels(L):
            got = u64(hb.hash_fixed(keys, L, seed=c["seed"], kernel=k) if L else
                      hb.hash_fixed(keys[:0], 0, seed=c["seed"], kernel=k))
            if L == 0:
                assert got.shape[0] == 0
                continue
            assert np.array_equal(got[0], want), (c["name"], k)
        # the same key through the variable-length path
        off = d_off(np.array([0, L], dtype=np.uint64), dev)
        for k in VAR_KERNELS:
            got = u64(hb.hash_var(keys, off, seed=c["seed"], kernel=k))
            assert np.array_equal(got[0], want), (c["name"], k)


@pytest.mark.parametrize("shift", [0, 1, 2, 3, 5, 8, 15])
def test_var_golden_any_alignment(hb, dev, golden_var, shift):
    data = np.concatenate([np.full(shift, 0xA5, np.uint8), golden_var["bytes"], np.full(3, 0x5A, np.uint8)])
    off = golden_var["offsets"] + np.uint64(shift)
    for k in VAR_KERNELS:
        got = u64(hb.hash_var(d_u8(data, dev), d_off(off, dev), kernel=k))
        assert np.array_equal(got, golden_var["hashes"]), k


@pytest.mark.parametrize("width", [4, 16])
def test_counter_keys_test9_shape(hb, dev, golden, width):
    g = golden["counters"]["counter_w%d" % width]
    keys = d_u8(counter_keys(g["count"], width), dev)
    for k in fixed_kernels(width):
        got = u64(hb.hash_fixed(keys, width, kernel=k))
        assert hashlib.sha256(got.astype("<u8").tobytes()).hexdigest() == g["sha256_of_hashes"], k


@pytest.mark.parametrize("name", ["fixed_w16", "fixed_w256"])
def test_fixed_random_golden(hb, dev, golden, name):
    g = golden["fixed"][name]
    flat = np.frombuffer(splitmix_bytes(g["key_len"] * g["count"], int(g["splitmix_stream"], 16)), dtype=np.uint8)
    keys = d_u8(flat, dev)
    for k in fixed_kernels(g["key_len"]):
        got = u64(hb.hash_fixed(keys, g["key_len"], kernel=k))
        assert hashlib.sha256(got.astype("<u8").tobytes()).hexdigest() == g["sha256_of_hashes"], k


# ---------------------------------------------------------------------------
# oracle parity over shapes and edge cases
# ---------------------------------------------------------------------------
LENGTHS = list(range(0, 81)) + [95, 96, 97, 112, 127, 128, 129, 144, 160, 240, 255, 256, 257, 272, 384, 511, 512,
                                528, 1024, 1040, 4096]


@pytest.mark.parametrize("n", [1, 63, 64, 65, 1000])
def test_fixed_all_lengths_all_kernels(hb, dev, oracle, n):
    rng = np.random.default_rng(n)
    for L in LENGTHS:
        if L == 0:
            continue
        flat = rng.integers(0, 256, size=n * L, dtype=np.uint8)
        want = oracle.hash_fixed(flat, L)
        keys = d_u8(flat, dev)
        for k in fixed_kernels(L):
            got = u64(hb.hash_fixed(keys, L, kernel=k))
            assert np.array_equal(got, want), (L, n, k)


def test_zero_length_keys(hb, dev, oracle):
    want = oracle.hash(b"")
    keys = torch.zeros(16, dtype=torch.uint8, device=dev)
    out = torch.zeros((5, 2), dtype=torch.int64, device=dev)
    rc = hb.load().shf_hash_batch_fixed_async(keys.data_ptr(), 0, 5, 12345, out.data_ptr(), None)
    assert rc == 0
    got = u64(out)
    assert all(tuple(int(x) for x in r) == want for r in got)
    off = d_off(np.zeros(6, dtype=np.uint64), dev)
    got = u64(hb.hash_var(keys, off))
    assert all(tuple(int(x) for x in r) == want for r in got)


@pytest.mark.parametrize("shift", [1, 2, 3, 4, 7, 13])
def test_fixed_unaligned_buffer(hb, dev, oracle, shift):
    rng = np.random.default_rng(shift)
    for L in [16, 32, 100, 256]:
        n = 777
        flat = rng.integers(0, 256, size=n * L + shift, dtype=np.uint8)
        want = oracle.hash_fixed(flat[shift:], L)
        keys = d_u8(flat, dev)[shift:]
        got = u64(hb.hash_fixed(keys, L))  # AUTO must notice the misalignment
        assert np.array_equal(got, want), (L, shift)


def test_var_random_lengths(hb, dev, oracle):
    rng = np.random.default_rng(7)
    for lo, hi, n in [(0, 16, 5000), (8, 512, 20000), (0, 2000, 3000), (500, 5000, 300)]:
        lens = rng.integers(lo, hi + 1, size=n)
        off = np.zeros(n + 1, dtype=np.uint64)
        off[1:] = np.cumsum(lens)
        data = rng.integers(0, 256, size=int(off[-1]) + 1, dtype=np.uint8)
        want = oracle.hash_var(data, off)
        for k in VAR_KERNELS:
            got = u64(hb.hash_var(d_u8(data, dev), d_off(off, dev), kernel=k))
            assert np.array_equal(got, want), (lo, hi, k)


def test_var_span_edges(hb, dev, oracle):
    """Tiles with no bytes, tiles exactly filling / overflowing the 20 KiB LDS
    window (global fallback), a last partial tile, buffers ending on a page."""
    rng = np.random.default_rng(17)
    cases = [
        np.zeros(200, dtype=np.int64),                                 # every tile empty
        np.concatenate([np.zeros(64, np.int64), rng.integers(0, 40, 100)]),
        np.full(64, 319, dtype=np.int64),                              # 20416 B: exactly the window
        np.full(64, 318, dtype=np.int64),
        np.full(64, 320, dtype=np.int64),                              # just over: direct from HBM
        np.full(130, 321, dtype=np.int64),                             # > window: fallback tiles
        np.concatenate([np.full(63, 1, np.int64), [20000], np.full(65, 7, np.int64)]),
        rng.integers(300, 340, size=1000),                             # straddles the window size
    ]
    for lens in cases:
        off = np.zeros(lens.size + 1, dtype=np.uint64)
        off[1:] = np.cumsum(lens)
        data = rng.integers(0, 256, size=max(int(off[-1]), 1), dtype=np.uint8)
        want = oracle.hash_var(data, off)
        # place the bytes so the buffer ends exactly at the end of a 4 KiB-aligned allocation
        pad = (-int(off[-1])) % 4096
        big = torch.zeros(pad + max(int(off[-1]), 1), dtype=torch.uint8, device=dev)
        big[pad:pad + int(off[-1])] = torch.from_numpy(data[:int(off[-1])]).to(dev)
        for k in VAR_KERNELS:
            got = u64(hb.hash_var(big, d_off(off + np.uint64(pad), dev), kernel=k))
            assert np.array_equal(got, want), (lens[:3], k)


def test_var_length_patterns(hb, dev, oracle):
    """Length patterns across tiles: all keys equal, rising and falling
    lengths, a mix of tiny and ~1-2 KB keys (tiles over the span window next to
    staged ones), 128- and 256-key batches of equal keys (whole tiles near the
    window size), a ragged batch ending in empty keys."""
    rng = np.random.default_rng(41)
    cases = [
        np.full(1000, 100, np.int64),
        np.arange(0, 1024, dtype=np.int64) % 700,
        np.arange(1024, 0, -1, dtype=np.int64) % 700,
        rng.choice([0, 1, 15, 16, 17, 1007, 1008, 1009, 2000], size=3000),
        np.full(128, 305, np.int64),
        np.full(128, 306, np.int64),
        np.full(256, 152, np.int64),
        np.concatenate([rng.integers(0, 600, 500), np.zeros(77, np.int64)]),
    ]
    for lens in cases:
        off = np.zeros(lens.size + 1, dtype=np.uint64)
        off[1:] = np.cumsum(lens)
        data = rng.integers(0, 256, size=max(int(off[-1]), 1), dtype=np.uint8)
        want = oracle.hash_var(data, off)
        for k in VAR_KERNELS:
            got = u64(hb.hash_var(d_u8(data, dev), d_off(off, dev), kernel=k))
            assert np.array_equal(got, want), (lens[:3], k)


@pytest.mark.parametrize("lo,hi", [(0, 40), (8, 128), (64, 192), (8, 256), (8, 512), (250, 330), (8, 2048)])
def test_var_sized_window(hb, dev, oracle, lo, hi):
    """shf_hash_batch_var_sized_*: the batch's byte count sizes the LDS window
    (10-20 KiB); the right count, a far too small one (every tile overflows
    into the round path) and a far too large one give the same hashes."""
    rng = np.random.default_rng(lo * 7 + hi)
    n = 30_000
    lens = rng.integers(lo, hi + 1, size=n)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    data = np.frombuffer(splitmix_bytes(int(off[-1]) + 5, lo + hi), dtype=np.uint8)[5:]
    want = oracle.hash_var(data, off)
    d_data, d_o = d_u8(data, dev), d_off(off, dev)
    total = int(off[-1])
    for kb in (total, 1, total * 50):
        for k in VAR_KERNELS:
            got = u64(hb.hash_var(d_data, d_o, kernel=k, key_bytes=kb))
            assert np.array_equal(got, want), (kb, k)
    lib = hb.load()
    out = torch.empty((n, 2), dtype=torch.int64, device=dev)
    assert lib.shf_hash_batch_var_sized_async(d_data.data_ptr(), d_o.data_ptr(), n, total, 12345, out.data_ptr(),
                                              None) == 0
    assert np.array_equal(u64(out), want)


def test_var_many_tiles(hb, dev, oracle):
    """A large batch (23k tiles) with a few tiles over the LDS window in between."""
    rng = np.random.default_rng(23)
    n = 1_500_000
    lens = rng.integers(0, 64, size=n)
    lens[rng.integers(0, n, size=300)] = 5000  # a few tiles overflow the window
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    data = rng.integers(0, 256, size=int(off[-1]), dtype=np.uint8)
    want = oracle.hash_var(data, off)
    d_data, d_o = d_u8(data, dev), d_off(off, dev)
    for k in VAR_KERNELS:
        assert np.array_equal(u64(hb.hash_var(d_data, d_o, kernel=k)), want), k
    # fixed lengths through the span kernel, many tiles per workgroup
    flat = rng.integers(0, 256, size=2_000_000 * 37, dtype=np.uint8)
    got = u64(hb.hash_fixed(d_u8(flat, dev), 37, kernel=4))
    assert np.array_equal(got, oracle.hash_fixed(flat, 37))


def test_var_many_oversized_tiles(hb, dev, oracle):
    """Half of the tiles too large for the LDS window (hashed from HBM), mixed
    with staged tiles."""
    rng = np.random.default_rng(29)
    n = 64 * 3000 * 4
    lens = rng.integers(0, 40, size=n)
    big = rng.random(n // 64) < 0.5  # half of the tiles get one 25 KB key
    lens[np.nonzero(big)[0] * 64 + 5] = 25000
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    data = rng.integers(0, 256, size=int(off[-1]), dtype=np.uint8)
    want = oracle.hash_var(data, off)
    for k in VAR_KERNELS:
        assert np.array_equal(u64(hb.hash_var(d_u8(data, dev), d_off(off, dev), kernel=k)), want), k


def test_var_near_window_and_deferred_mixed(hb, dev, oracle):
    """Spans straddling the LDS window: staged tiles that use the window's last
    1 KiB piece (partially) interleaved with tiles hashed from HBM."""
    rng = np.random.default_rng(31)
    n = 64 * 30000
    lens = rng.integers(308, 330, size=n)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    data = rng.integers(0, 256, size=int(off[-1]), dtype=np.uint8)
    want = oracle.hash_var(data, off)
    got = u64(hb.hash_var(d_u8(data, dev), d_off(off, dev), kernel=4))
    assert np.array_equal(got, want)


@pytest.mark.parametrize("shift", [0, 5, 13])
def test_var_round_edges(hb, dev, oracle, shift):
    """k_vround: keys at the staged-path limit (8192 B = 64 rounds) and just past
    it (HBM fallback), lengths 0..17 and 127..129 around round and piece
    boundaries, empty keys at the very end of the buffer, unaligned starts."""
    rng = np.random.default_rng(77 + shift)
    pieces = []
    for _ in range(3000):
        pieces.append(rng.choice([0, 1, 15, 16, 17, 127, 128, 129, 143, 144, 145, 255, 256, 257]))
    lens = np.array(pieces, dtype=np.uint64)
    lens[640:704] = rng.choice([8175, 8176, 8177, 8191, 8192], size=64)  # one tile at the limit
    lens[1280] = 8193  # this tile falls back
    lens[-5:] = 0  # empty keys at the end
    off = np.zeros(lens.size + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    data = np.frombuffer(splitmix_bytes(int(off[-1]) + shift, 5 + shift), dtype=np.uint8)
    want = oracle.hash_var(data[shift:], off)
    got = u64(hb.hash_var(d_u8(data, dev), d_off(off + np.uint64(shift), dev), kernel=5))
    assert np.array_equal(got, want)


def test_var_long_keys(hb, dev, oracle):
    lens = np.array([65537, 1 << 20, 3, (1 << 20) + 15, 0, 100000], dtype=np.uint64)
    off = np.zeros(lens.size + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    data = np.frombuffer(splitmix_bytes(int(off[-1]), 99), dtype=np.uint8)
    want = oracle.hash_var(data, off)
    for k in VAR_KERNELS:
        got = u64(hb.hash_var(d_u8(data, dev), d_off(off, dev), kernel=k))
        assert np.array_equal(got, want), k


@pytest.mark.parametrize("lo,hi", [(8, 2048), (400, 1200)])
def test_var_long_keys_without_byte_count(hb, dev, oracle, lo, hi):
    """Keys whose 64-key spans overflow the 20-KiB window, hashed without a
    byte count (AUTO -> k_span_pp) and through SHF_HB_KERNEL_SPAN_PP: the
    overflowing tiles are streamed through the window in rounds in their
    wave's turn (they used to be hashed per lane from HBM)."""
    rng = np.random.default_rng(lo + hi)
    n = 64 * 700 + 13
    lens = rng.integers(lo, hi + 1, size=n)
    lens[64 * 5 + 3] = 9000  # a key past the round path's 8 KiB: that tile per lane from HBM
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    data = rng.integers(0, 256, size=int(off[-1]) + 5, dtype=np.uint8)
    want = oracle.hash_var(data, off)
    d_data, d_o = d_u8(data, dev), d_off(off, dev)
    for k in (0, 6):
        assert np.array_equal(u64(hb.hash_var(d_data, d_o, kernel=k)), want), k
    # shifted start: every key unaligned
    d_o3 = d_off(off + np.uint64(3), dev)
    for k in (6,):
        assert np.array_equal(u64(hb.hash_var(d_data, d_o3, kernel=k)), oracle.hash_var(data[3:], off)), k


@pytest.mark.parametrize("base", [(1 << 31) + 12345, (1 << 32) + 12345, (3 << 31) + 7])
def test_var_offsets_beyond_2gib(hb, dev, oracle, base):
    """64-bit offsets: keys living past 2 GiB / 4 GiB of the byte buffer, with
    bit 31 of the low offset word set and clear (no sign extension anywhere)."""
    n = 2000
    rng = np.random.default_rng(3)
    lens = rng.integers(0, 300, size=n)
    rel = np.zeros(n + 1, dtype=np.uint64)
    rel[1:] = np.cumsum(lens)
    payload = rng.integers(0, 256, size=int(rel[-1]), dtype=np.uint8)
    big = torch.empty(base + int(rel[-1]) + 64, dtype=torch.uint8, device=dev)
    big[base:base + payload.size] = torch.from_numpy(payload).to(dev)
    want = oracle.hash_var(payload, rel)
    for k in VAR_KERNELS:
        got = u64(hb.hash_var(big, d_off(rel + np.uint64(base), dev), kernel=k))
        assert np.array_equal(got, want), k
    del big
    torch.cuda.empty_cache()


def test_seeds(hb, dev, oracle):
    rng = np.random.default_rng(11)
    flat = rng.integers(0, 256, size=300 * 48, dtype=np.uint8)
    keys = d_u8(flat, dev)
    for seed in [0, 1, 12345, 0x7FFFFFFF, 0x80000000, 0xFFFFFFFF]:
        for k in fixed_kernels(48):
            got = u64(hb.hash_fixed(keys, 48, seed=seed, kernel=k))
            assert np.array_equal(got, oracle.hash_fixed(flat, 48, seed=seed)), (seed, k)


def test_uid_parts(hb, dev, oracle, golden_var):
    rng = np.random.default_rng(5)
    for L in [4, 16, 256, 37]:
        flat = rng.integers(0, 256, size=3000 * L, dtype=np.uint8)
        want = oracle.uid_parts(oracle.hash_fixed(flat, L))
        got = u64(hb.uid_parts_fixed(d_u8(flat, dev), L))
        assert np.array_equal(got, want), L
    got = u64(hb.uid_parts_var(d_u8(golden_var["bytes"], dev), d_off(golden_var["offsets"], dev)))
    assert np.array_equal(got, oracle.uid_parts(golden_var["hashes"]))


def test_async_on_side_stream(hb, dev, oracle):
    rng = np.random.default_rng(8)
    flat = rng.integers(0, 256, size=100000 * 16, dtype=np.uint8)
    keys = d_u8(flat, dev)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        out = hb.hash_fixed(keys, 16, stream=s)
    s.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint64), oracle.hash_fixed(flat, 16))


# ---------------------------------------------------------------------------
# host-memory and multi-device entry points
# ---------------------------------------------------------------------------
def test_host_fixed_multi_chunk(hb, dev, oracle):
    n = 5_000_000  # 80 MB of 16-B keys: more than one 64 MiB staging chunk
    flat = np.frombuffer(splitmix_bytes(n * 16, 21), dtype=np.uint8)
    got = hb.hash_fixed_host(flat, 16)
    assert np.array_equal(got, oracle.hash_fixed(flat, 16, threads=8))
    got = hb.hash_fixed_host(flat, 16, n_devices=0)
    assert np.array_equal(got, oracle.hash_fixed(flat, 16, threads=8))


def test_host_var_multi_chunk(hb, dev, oracle):
    rng = np.random.default_rng(12)
    n = 300_000
    lens = rng.integers(8, 513, size=n)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)  # ~78 MB of key bytes
    data = rng.integers(0, 256, size=int(off[-1]), dtype=np.uint8)
    want = oracle.hash_var(data, off)
    assert np.array_equal(hb.hash_var_host(data, off), want)
    assert np.array_equal(hb.hash_var_host(data, off, n_devices=0), want)


@pytest.mark.parametrize("lo,hi", [(0, 40), (8, 128), (200, 400), (300, 3000)])
def test_host_var_kernel_by_mean_length(hb, dev, oracle, lo, hi):
    """The host path sizes the span kernel's window by each chunk's mean key
    length, and takes the round kernel past a mean of 300 B."""
    rng = np.random.default_rng(lo + hi)
    n = 40_000
    lens = rng.integers(lo, hi + 1, size=n)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    data = np.frombuffer(splitmix_bytes(int(off[-1]) + 3, lo + 1), dtype=np.uint8)[3:]
    assert np.array_equal(hb.hash_var_host(data, off), oracle.hash_var(data, off))


@pytest.mark.parametrize("stage_mb,slots,pool_mb", [(1, 2, 64), (1, 4, 64), (3, 3, 64), (64, 2, 256), (1, 4, 1),
                                                    (16, 4, 16), (2, 1, 64), (16, 4, 8)])
def test_host_pipeline_shapes(hb, dev, oracle, monkeypatch, stage_mb, slots, pool_mb):
    """SHF_HB_STAGE_MB / SHF_HB_SLOTS / SHF_HB_POOL_MB change only how a host
    batch is chunked and overlapped (many chunks, a key larger than a slot),
    down to a pool of one slot (pool smaller than one slot: still one)."""
    monkeypatch.setenv("SHF_HB_STAGE_MB", str(stage_mb))
    monkeypatch.setenv("SHF_HB_SLOTS", str(slots))
    monkeypatch.setenv("SHF_HB_POOL_MB", str(pool_mb))
    n = 600_000
    flat = np.frombuffer(splitmix_bytes(n * 16, 31), dtype=np.uint8)
    assert np.array_equal(hb.hash_fixed_host(flat, 16), oracle.hash_fixed(flat, 16, threads=8))
    rng = np.random.default_rng(stage_mb * 10 + slots)
    m = 20_000
    lens = rng.integers(0, 700, size=m)
    lens[5] = 3 << 20
    off = np.zeros(m + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    data = rng.integers(0, 256, size=int(off[-1]), dtype=np.uint8)
    assert np.array_equal(hb.hash_var_host(data, off), oracle.hash_var(data, off))


@pytest.mark.parametrize("direct_out", ["1", "0"])
def test_host_pinned_buffers(hb, dev, oracle, monkeypatch, direct_out):
    """Caller buffers already page-locked: DMA'd directly (no staging copy),
    the hashes stored by the kernel straight into the output (1) or copied
    back per chunk (SHF_HB_DIRECT_OUT=0)."""
    monkeypatch.setenv("SHF_HB_DIRECT_OUT", direct_out)
    lib = hb.load()
    n = 3_000_000
    keys = torch.randint(0, 256, (n * 16,), dtype=torch.uint8).pin_memory()
    out = torch.zeros((n, 2), dtype=torch.int64).pin_memory()
    rc = lib.shf_hash_batch_fixed(keys.data_ptr(), 16, n, 12345, out.data_ptr(), hb.MEM_HOST)
    assert rc == 0
    assert np.array_equal(out.numpy().view(np.uint64), oracle.hash_fixed(keys.numpy(), 16, threads=8))
    rng = np.random.default_rng(13)
    m = 200_000
    lens = rng.integers(0, 600, size=m)
    off = torch.zeros(m + 1, dtype=torch.int64).pin_memory()
    off[1:] = torch.from_numpy(np.cumsum(lens))
    data = torch.randint(0, 256, (int(off[-1]),), dtype=torch.uint8).pin_memory()
    out2 = torch.zeros((m, 2), dtype=torch.int64).pin_memory()
    rc = lib.shf_hash_batch_var(data.data_ptr(), off.data_ptr(), m, 12345, out2.data_ptr(), hb.MEM_HOST)
    assert rc == 0
    assert np.array_equal(out2.numpy().view(np.uint64), oracle.hash_var(data.numpy(), off.numpy().view(np.uint64)))


@pytest.mark.parametrize("key_len", [1, 7, 16, 24, 32, 33, 128, 129])
def test_host_zero_copy(hb, dev, oracle, monkeypatch, key_len):
    """Page-locked caller buffers, keys up to SHF_HB_ZERO_COPY_MAX_KEY: the
    kernel reads keys and writes hashes over PCIe itself. Interior pointers
    (unaligned keys, an output that starts past the allocation's first record),
    the staged path forced (0), and a pageable output (staged) give the same
    bits as the oracle."""
    lib = hb.load()
    n = 100_003
    pad = 5
    keys = torch.randint(0, 256, (n * key_len + 2 * pad,), dtype=torch.uint8).pin_memory()
    flat = keys.numpy()[pad:pad + n * key_len]
    want = oracle.hash_fixed(flat, key_len, threads=8)
    for env in ("32", "0", "1048576"):
        monkeypatch.setenv("SHF_HB_ZERO_COPY_MAX_KEY", env)
        out = torch.zeros((n + 3, 2), dtype=torch.int64).pin_memory()
        rc = lib.shf_hash_batch_fixed(keys.data_ptr() + pad, key_len, n, 12345, out.data_ptr() + 48, hb.MEM_HOST)
        assert rc == 0
        assert np.array_equal(out.numpy().view(np.uint64)[3:], want), env
        assert not out.numpy()[:3].any()
    pageable = np.zeros((n, 2), dtype=np.uint64)
    assert lib.shf_hash_batch_fixed(keys.data_ptr() + pad, key_len, n, 12345, pageable.ctypes.data, hb.MEM_HOST) == 0
    assert np.array_equal(pageable, want)
    one = torch.zeros((1, 2), dtype=torch.int64).pin_memory()  # a single key
    assert lib.shf_hash_batch_fixed(keys.data_ptr() + pad, key_len, 1, 12345, one.data_ptr(), hb.MEM_HOST) == 0
    assert np.array_equal(one.numpy().view(np.uint64), want[:1])


def test_multi_shards_share_boundary_pages(hb, dev, oracle, monkeypatch):
    """*_multi shards over one pageable buffer, split mid-page: each shard
    locks only the pages wholly inside its own key and hash ranges, so the
    page two shards share is locked by neither and both reach it through the
    staged pipeline (SHF_HB_MULTI_SHARE_DEVICES: the shards' threads share one
    GPU here)."""
    monkeypatch.setenv("SHF_HB_MULTI_SHARE_DEVICES", "1")
    lib = hb.load()
    n = 1_000_003  # shard boundaries at n * d / g: mid-page for g = 2, 3, 5
    flat = np.frombuffer(splitmix_bytes(n * 16, 43), dtype=np.uint8).copy()
    want = oracle.hash_fixed(flat, 16, threads=8)
    for g in (2, 3, 5):
        out = np.zeros((n, 2), dtype=np.uint64)
        assert lib.shf_hash_batch_fixed_multi(flat.ctypes.data, 16, n, 12345, out.ctypes.data, g) == 0, g
        assert np.array_equal(out, want), g


def test_host_huge_single_key(hb, dev, oracle):
    n_big = (70 << 20) + 9  # one key larger than a staging chunk
    data = np.frombuffer(splitmix_bytes(n_big + 100, 5), dtype=np.uint8)
    off = np.array([0, 50, 50 + n_big, n_big + 100], dtype=np.uint64)
    assert np.array_equal(hb.hash_var_host(data, off), oracle.hash_var(data, off))


# ---------------------------------------------------------------------------
# full-size properties (bench shapes): kernels agree, sampled oracle parity
# ---------------------------------------------------------------------------
def _sample_check(oracle, keys_dev, L, got, count=20000, seed=0):
    n = got.shape[0]
    idx = np.unique(np.random.default_rng(seed).integers(0, n, size=count))
    rows = keys_dev.view(-1, L)[torch.from_numpy(idx).to(keys_dev.device)].cpu().numpy()
    assert np.array_equal(got[idx], oracle.hash_fixed(rows, L))


def test_config_b_10m_16b(hb, dev, oracle):
    n, L = 10_000_000, 16
    keys = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device=dev)
    a = hb.hash_fixed(keys, L, kernel=1)
    b = hb.hash_fixed(keys, L, kernel=3)
    assert torch.equal(a, b)
    _sample_check(oracle, keys, L, u64(a))
    # uid parts are a function of the hash (shf.c:800-803)
    p = hb.uid_parts_fixed(keys, L)
    h1, h2 = a[:, 0], a[:, 1]
    want = (h1 & 0xFF) | (((h1 >> 16) & 0x7FF) << 8) | (((h1 >> 32) & 0x1FF) << 19) | ((h2 & 0x1FFFFF) << 32)
    assert torch.equal(p, want)


def test_256b_kernels_agree(hb, dev, oracle):
    n, L = 2_000_003, 256
    keys = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device=dev)
    a = hb.hash_fixed(keys, L, kernel=2)
    b = hb.hash_fixed(keys, L, kernel=3)
    assert torch.equal(a, b)
    _sample_check(oracle, keys, L, u64(a))
