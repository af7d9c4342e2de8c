"""The pageable zero copy (on by default,
SHF_HB_PAGEABLE_ZERO_COPY=0 turns it off): the whole pages of a pageable caller
buffer are page-locked for one call and read / written by the kernel over PCIe.

In round 4 two full GPU test runs with it on failed later, in an unrelated
pageable copy of the same process; the test then moved to a file that ran
last. tools/pageable_register_repro.hip reproduces that exact error only from a
registration that outlives the memory it covers, the library
now checks every lock and unlock against the runtime, and this file runs with
the other GPU tests (early: test_gpu_h* sorts before the parity suites), each
of which takes the path by default. The last test below checks, after many
calls, that every page the library locked is unlocked again and that a fresh
buffer at a reused address copies cleanly."""
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


@pytest.mark.parametrize("key_len,kpad,opad", [(16, 0, 0), (16, 48, 16), (24, 7, 32), (100, 4093, 4080)])
def test_host_pageable_zero_copy(hb, dev, oracle, monkeypatch, key_len, kpad, opad):
    """Pageable caller buffers: the pages wholly inside the key and hash
    ranges are page-locked for the call and read / written by the kernel over
    PCIe, the keys at the ends go through the staged pipeline. Interior
    offsets put the range ends mid-page (and unaligned keys on k_generic); the
    same bits as the oracle with the path on, off, and with nothing beside
    the caller's range touched."""
    lib = hb.load()
    n = 300_007
    kbuf = np.frombuffer(splitmix_bytes(n * key_len + kpad + 64, 41 + key_len), dtype=np.uint8).copy()
    flat = kbuf[kpad:kpad + n * key_len]
    want = oracle.hash_fixed(flat, key_len, threads=8)
    for env in ("1", "0", None):
        if env is None:
            monkeypatch.delenv("SHF_HB_PAGEABLE_ZERO_COPY", raising=False)  # the default: on
        else:
            monkeypatch.setenv("SHF_HB_PAGEABLE_ZERO_COPY", env)
        obuf = np.zeros(n * 16 + opad + 64, dtype=np.uint8)
        rc = lib.shf_hash_batch_fixed(kbuf.ctypes.data + kpad, key_len, n, 12345, obuf.ctypes.data + opad,
                                      hb.MEM_HOST)
        assert rc == 0, env
        got = obuf[opad:opad + n * 16].view(np.uint64).reshape(n, 2)
        assert np.array_equal(got, want), env
        assert not obuf[:opad].any() and not obuf[opad + n * 16:].any(), env
    # the buffers are pageable again afterwards (each call unlocked what it locked)
    assert lib.shf_hash_batch_fixed(kbuf.ctypes.data + kpad, key_len, n, 12345, obuf.ctypes.data + opad,
                                    hb.MEM_HOST) == 0


def test_locked_pages_are_released_and_reused_addresses_copy_cleanly(hb, dev, oracle, monkeypatch):
    """The round-4 failure's shape, done on purpose: pageable buffers of one size
    are hashed through the zero copy (their pages locked and unlocked), freed,
    and buffers of the same size, which glibc places at the same addresses, are
    then copied by torch's pageable .to(device) -- 1,600,048 B like both failing
    copies. Afterwards the runtime resolves none of the pages the library locked."""
    import ctypes

    monkeypatch.delenv("SHF_HB_PAGEABLE_ZERO_COPY", raising=False)
    lib = hb.load()
    n = 100_003
    addrs = []
    for r in range(12):
        keys = np.frombuffer(splitmix_bytes(n * 16, 300 + r), dtype=np.uint8).copy()
        out = np.empty((n, 2), dtype=np.uint64)
        assert lib.shf_hash_batch_fixed(keys.ctypes.data, 16, n, 12345, out.ctypes.data, hb.MEM_HOST) == 0
        assert np.array_equal(out[:: 997], oracle.hash_fixed(keys.reshape(n, 16)[:: 997], 16))
        addrs += [keys.ctypes.data, out.ctypes.data]
        del keys, out
        fresh = np.frombuffer(splitmix_bytes(n * 16, 400 + r), dtype=np.uint8).copy()
        t = torch.from_numpy(fresh).to(dev)
        torch.cuda.synchronize()
        assert np.array_equal(t.cpu().numpy(), fresh)
    # no page the library locked is still resolved by the runtime
    still = [a for a in addrs if _runtime_registered(a + 8192)]
    assert not still, [hex(a) for a in still]


def _runtime_registered(addr):
    """hipPointerGetAttributes(addr).type == hipMemoryTypeHost (the runtime resolves
    the host address to a device mapping), asked of the HIP runtime torch loaded."""
    import ctypes

    hip = ctypes.CDLL("libamdhip64.so", mode=ctypes.RTLD_GLOBAL)
    attr = (ctypes.c_int * 64)()  # hipPointerAttribute_t starts with its hipMemoryType
    rc = hip.hipPointerGetAttributes(ctypes.byref(attr), ctypes.c_void_p(addr))
    if rc != 0:
        hip.hipGetLastError()
        return False
    return attr[0] == 1  # hipMemoryTypeHost
