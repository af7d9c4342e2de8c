"""Deterministic synthetic key generators (SURVEY.md s8(d) "Synthetic inputs").

Key bytes come from splitmix64 streams, so host (numpy) and device (torch)
generators produce the same bytes for the same stream id, and the golden
fixtures can name their inputs by stream id.
"""
import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix_u64(count: int, stream: int, start: int = 0) -> np.ndarray:
    """Values start..start+count-1 of the splitmix64 sequence seeded `stream`."""
    with np.errstate(over="ignore"):
        idx = np.arange(start + 1, start + count + 1, dtype=np.uint64)
        z = np.uint64(stream & 0xFFFFFFFFFFFFFFFF) + idx * _GOLDEN
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def splitmix_bytes(nbytes: int, stream: int) -> bytes:
    words = splitmix_u64((nbytes + 7) // 8, stream)
    return words.astype("<u8").tobytes()[:nbytes]


def splitmix_lengths(count: int, lo: int, hi: int, stream: int) -> np.ndarray:
    """count lengths uniform-ish in [lo, hi] (modulo reduction of splitmix64)."""
    span = np.uint64(hi - lo + 1)
    return (splitmix_u64(count, stream) % span).astype(np.int64) + lo


def counter_keys(count: int, key_len: int, first: int = 0) -> np.ndarray:
    """test.9-style keys: the little-endian bytes of uint32 i, zero-padded to
    key_len (src/test.9.shf.c:429 hashes the 4 bytes of `uint32_t i`)."""
    keys = np.zeros((count, key_len), dtype=np.uint8)
    ctr = np.arange(first, first + count, dtype="<u4").view(np.uint8).reshape(count, 4)
    w = min(4, key_len)
    keys[:, :w] = ctr[:, :w]
    return keys


def device_random_bytes(nbytes: int, seed: int, device):
    """Large random key buffers generated on the GPU (torch's Philox, seeded).
    Used by bench.py where host generation of tens of GB would dominate."""
    import torch

    g = torch.Generator(device=device)
    g.manual_seed(seed)
    out = torch.empty(nbytes, dtype=torch.uint8, device=device)
    chunk = 1 << 30
    for s in range(0, nbytes, chunk):
        e = min(nbytes, s + chunk)
        out[s:e].random_(0, 256, generator=g)
    return out
