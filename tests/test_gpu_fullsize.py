"""Full-size parity at BASELINE.json's bench shapes.

The batches bench.py times are too large for the oracle, so each is checked
through size-independent properties: every kernel that accepts the shape gives
the same 128 bits for every key (torch.equal over the whole batch), and 20 000
sampled keys plus the first and the last match the oracle (oracle/, the C
restatement pinned to the reference's goldens by tests/test_oracle.py).

  configs[2]  100M x 256 B      (25.6 GB)  AUTO (k_tiled), k_tiled, k_generic
  configs[3]  100M x U[8,512] B (~26 GB)   AUTO, k_span, k_vround, k_generic, k_span_pp
  configs[4]  1B x 16 B         (16 GB)    AUTO (k_fixed16), k_fixed16, k_generic

and the same three shapes through the host-memory pipeline from pageable
buffers (every key against the device kernels, a sample against the oracle).

Runs only on a real MI355X: python -m pytest tests -m gpu
"""
import numpy as np
import pytest

from sharedhashfile_amd.keygen import device_random_bytes

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev(hb):
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    hb.check_device()  # raises unless the current device is gfx950
    return torch.device("cuda:0")


def _sample(n, seed, count=20000):
    idx = np.random.default_rng(seed).integers(0, n, size=count)
    return np.unique(np.concatenate([idx, [0, n - 1]]))


def _u64(t):
    torch.cuda.synchronize()
    return t.cpu().numpy().view(np.uint64)


def _fixed_case(hb, dev, oracle, n, key_len, kernels, seed):
    keys = device_random_bytes(n * key_len, seed, dev)
    ref = hb.hash_fixed(keys, key_len, kernel=kernels[0])
    for k in kernels[1:]:
        out = hb.hash_fixed(keys, key_len, kernel=k)
        assert torch.equal(out, ref), "kernel %d differs from kernel %d" % (k, kernels[0])
        del out
    idx = _sample(n, seed)
    ti = torch.from_numpy(idx).to(dev)
    rows = keys.view(n, key_len)[ti].cpu().numpy()
    assert np.array_equal(_u64(ref[ti]), oracle.hash_fixed(rows, key_len))


def test_config2_100m_256b(hb, dev, oracle):
    _fixed_case(hb, dev, oracle, 100_000_000, 256, [0, 2, 3], 21)


def test_config4_1b_16b(hb, dev, oracle):
    _fixed_case(hb, dev, oracle, 1_000_000_000, 16, [0, 1, 3], 22)


def test_config3_100m_var(hb, dev, oracle):
    n = 100_000_000
    g = torch.Generator(device=dev)
    g.manual_seed(23)
    lens = torch.randint(8, 513, (n,), generator=g, device=dev, dtype=torch.int64)
    off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    torch.cumsum(lens, 0, out=off[1:])
    del lens
    data = device_random_bytes(int(off[-1].item()), 24, dev)
    ref = hb.hash_var(data, off, kernel=0)
    for k in (4, 5, 3, 6):  # SPAN, ROUND, GENERIC, SPAN_PP
        out = hb.hash_var(data, off, kernel=k)
        assert torch.equal(out, ref), "kernel %d differs from AUTO" % k
        del out
    idx = _sample(n, 23)
    ti = torch.from_numpy(idx).to(dev)
    so, ln = off[ti], off[ti + 1] - off[ti]
    sub_off = torch.zeros(len(idx) + 1, dtype=torch.int64, device=dev)
    torch.cumsum(ln, 0, out=sub_off[1:])
    gather = torch.repeat_interleave(so - sub_off[:-1], ln) + torch.arange(int(sub_off[-1].item()), device=dev)
    sub = data[gather].cpu().numpy()
    want = oracle.hash_var(sub, sub_off.cpu().numpy().view(np.uint64))
    assert np.array_equal(_u64(ref[ti]), want)


# The host-memory pipeline (SHF_HASH_MEM_HOST) at the same full sizes, from
# pageable buffers: thousands of chunks through the process's staging slots,
# byte positions far past 2^32, fixed-length keys through the runtime's
# pageable copy and variable-length ones staged on the CPU. Every key's 128 bits
# against the device kernels' (compared on the device), plus a sample against
# the oracle straight from the host bytes.
def _host_against(got, ref, dev):
    assert got.shape == tuple(ref.shape)
    assert torch.equal(torch.from_numpy(got.view(np.int64)).to(dev), ref)


def _host_fixed_case(hb, dev, oracle, n, key_len, seed):
    keys = device_random_bytes(n * key_len, seed, dev)
    ref = hb.hash_fixed(keys, key_len)
    host = keys.cpu().numpy()  # pageable
    del keys
    got = hb.hash_fixed_host(host, key_len)
    _host_against(got, ref, dev)
    idx = _sample(n, seed, 2000)
    assert np.array_equal(got[idx], oracle.hash_fixed(host.reshape(n, key_len)[idx], key_len))


def test_host_config2_100m_256b(hb, dev, oracle):
    _host_fixed_case(hb, dev, oracle, 100_000_000, 256, 25)


def test_host_config4_1b_16b(hb, dev, oracle):
    _host_fixed_case(hb, dev, oracle, 1_000_000_000, 16, 26)


def test_host_config3_100m_var(hb, dev, oracle):
    n = 100_000_000
    g = torch.Generator(device=dev)
    g.manual_seed(27)
    lens = torch.randint(8, 513, (n,), generator=g, device=dev, dtype=torch.int64)
    off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    torch.cumsum(lens, 0, out=off[1:])
    del lens
    data = device_random_bytes(int(off[-1].item()), 28, dev)
    ref = hb.hash_var(data, off)
    h_data, h_off = data.cpu().numpy(), off.cpu().numpy().view(np.uint64)
    del data, off
    got = hb.hash_var_host(h_data, h_off)
    _host_against(got, ref, dev)
    idx = _sample(n, 27, 2000)
    sub_off = np.zeros(len(idx) + 1, dtype=np.uint64)
    sub_off[1:] = np.cumsum(h_off[idx + 1] - h_off[idx])
    sub = np.concatenate([h_data[h_off[i]:h_off[i + 1]] for i in idx])
    assert np.array_equal(got[idx], oracle.hash_var(sub, sub_off))
