"""Pageable caller buffers (SHF_HASH_MEM_HOST): the library never page-locks
them; they go through the staged pipeline.

Rounds 3-5 had a pageable zero copy (the buffer's whole interior pages
registered for one call and read / written by the kernel over PCIe). With it
on, 3 of the last 5 full GPU test runs failed later in an unrelated pageable
copy of the test process (torch's .to(device) / .cpu(), hipErrorIllegalAddress),
none of 6 with it off; tools/pageable_register_repro.hip shows that error comes from a
registration outliving its memory. The path is gone. These
tests pin what replaced it: the same bits from pageable buffers at any offset,
nothing beside the caller's range touched, no page of a caller buffer left
registered with the runtime, and the round-4 failure's shape -- buffers hashed,
freed, and fresh buffers at the same addresses copied by torch -- clean.
This file runs early among the GPU tests (test_gpu_h* sorts before the parity
suites), so anything it left behind would meet every later test.
"""
import ctypes

import numpy as np
import pytest

from sharedhashfile_amd.keygen import splitmix_bytes

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev(hb):
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    hb.check_device()
    return torch.device("cuda:0")


def _runtime_registered(addr):
    """hipPointerGetAttributes(addr).type == hipMemoryTypeHost: the runtime
    resolves the host address to a device mapping (asked of the HIP runtime
    torch loaded)."""
    hip = ctypes.CDLL("libamdhip64.so", mode=ctypes.RTLD_GLOBAL)
    attr = (ctypes.c_int * 64)()  # hipPointerAttribute_t starts with its hipMemoryType
    rc = hip.hipPointerGetAttributes(ctypes.byref(attr), ctypes.c_void_p(addr))
    if rc != 0:
        hip.hipGetLastError()
        return False
    return attr[0] == 1  # hipMemoryTypeHost


@pytest.mark.parametrize("key_len,kpad,opad", [(16, 0, 0), (16, 48, 16), (24, 7, 32), (100, 4093, 4080)])
def test_host_pageable_buffers(hb, dev, oracle, key_len, kpad, opad):
    """Pageable key and hash buffers at interior offsets (range ends mid-page,
    unaligned keys on k_generic): the same bits as the oracle, nothing beside
    the caller's range touched, and no page of either buffer registered with
    the runtime during or after the call."""
    lib = hb.load()
    n = 300_007
    kbuf = np.frombuffer(splitmix_bytes(n * key_len + kpad + 64, 41 + key_len), dtype=np.uint8).copy()
    flat = kbuf[kpad:kpad + n * key_len]
    want = oracle.hash_fixed(flat, key_len, threads=8)
    obuf = np.zeros(n * 16 + opad + 64, dtype=np.uint8)
    rc = lib.shf_hash_batch_fixed(kbuf.ctypes.data + kpad, key_len, n, 12345, obuf.ctypes.data + opad, hb.MEM_HOST)
    assert rc == 0
    got = obuf[opad:opad + n * 16].view(np.uint64).reshape(n, 2)
    assert np.array_equal(got, want)
    assert not obuf[:opad].any() and not obuf[opad + n * 16:].any()
    for base, size in ((kbuf.ctypes.data, kbuf.size), (obuf.ctypes.data, obuf.size)):
        assert not any(_runtime_registered(a) for a in range(base, base + size, 1 << 16))


def test_reused_addresses_copy_cleanly(hb, dev, oracle):
    """The round-4 failure's shape, done on purpose: pageable buffers hashed
    through the library, freed, and buffers of the same size -- which glibc
    places at the same addresses -- then copied by torch's pageable
    .to(device) and .cpu(), 1,600,048 B like both round-4 failing copies."""
    lib = hb.load()
    n = 100_003
    for r in range(12):
        keys = np.frombuffer(splitmix_bytes(n * 16, 300 + r), dtype=np.uint8).copy()
        out = np.empty((n, 2), dtype=np.uint64)
        assert lib.shf_hash_batch_fixed(keys.ctypes.data, 16, n, 12345, out.ctypes.data, hb.MEM_HOST) == 0
        assert np.array_equal(out[::997], oracle.hash_fixed(keys.reshape(n, 16)[::997], 16))
        del keys, out
        fresh = np.frombuffer(splitmix_bytes(n * 16, 400 + r), dtype=np.uint8).copy()
        t = torch.from_numpy(fresh).to(dev)
        back = t.cpu().numpy()
        torch.cuda.synchronize()
        assert np.array_equal(back, fresh)


@pytest.mark.parametrize("runtime_h2d,copy_nt,threads,direct_out",
                         [("1", "1", "12", "1"), ("0", "1", "12", "1"), ("1", "0", "1", "1"), ("0", "0", "3", "0"),
                          ("1", "1", "2", "0")])
def test_host_pageable_copy_settings(hb, dev, oracle, monkeypatch, runtime_h2d, copy_nt, threads, direct_out):
    """Every way a pageable batch moves (read per call): keys through the
    runtime's pageable copy with the records copied out on the copy workers
    (SHF_HB_RUNTIME_H2D=1) or staged on the CPU (0), streaming stores or
    memcpy, 1-12 copy threads, records stored by the kernel into the slot or
    copied back. 1-MiB slots, three of them, so every chunk's copy-out runs
    beside a later chunk's copy-in; hashes, probe records and both at once,
    fixed (16 B: k_fixed16; 40 B: another kernel) and variable lengths."""
    from sharedhashfile_amd.keygen import splitmix_lengths
    from sharedhashfile_amd.rowindex import synthetic_index

    for k, v in (("SHF_HB_RUNTIME_H2D", runtime_h2d), ("SHF_HB_COPY_NT", copy_nt), ("SHF_HB_COPY_THREADS", threads),
                 ("SHF_HB_DIRECT_OUT", direct_out), ("SHF_HB_STAGE_MB", "1"), ("SHF_HB_SLOTS", "3")):
        monkeypatch.setenv(k, v)
    for key_len, n in ((16, 400_003), (40, 150_001)):
        flat = np.frombuffer(splitmix_bytes(n * key_len, 70 + key_len), dtype=np.uint8)
        want = oracle.hash_fixed(flat, key_len, threads=8)
        assert np.array_equal(hb.hash_fixed_host(flat, key_len), want)
    m = 60_000
    off = np.zeros(m + 1, dtype=np.uint64)
    off[1:] = np.cumsum(splitmix_lengths(m, 8, 512, 73))
    data = np.frombuffer(splitmix_bytes(int(off[-1]), 74), dtype=np.uint8)
    assert np.array_equal(hb.hash_var_host(data, off), oracle.hash_var(data, off))
    keys = np.frombuffer(splitmix_bytes(300_007 * 16, 75), dtype=np.uint8).reshape(-1, 16)
    h = oracle.hash_fixed(keys.reshape(-1), 16, threads=8)
    tab_slot, rows, n_slots, _ = synthetic_index(h, tabs_per_win=2, limit=len(h) - 1000)
    idx = hb.RowIndex(n_slots, tab_slot, rows)
    try:
        want = oracle.probe(h, tab_slot, rows)
        rec, hh = hb.probe_fixed_host(idx, keys, hashes=True)
        assert np.array_equal(rec, want) and np.array_equal(hh, h)
        assert np.array_equal(hb.probe_fixed_host(idx, keys), want)
    finally:
        idx.close()
