"""Key-range sharding across GPUs.

Keys are independent, so a batch splits into contiguous, even index ranges, one
per rank/GPU, with no collective on the data path. A variable-length batch
splits by key index too; each shard's bytes are the slice
bytes[offsets[lo] : offsets[hi]) and its offsets are rebased by offsets[lo]
(the kernels take absolute offsets, so rebasing is optional).

The same split is used by the C ABI's *_multi entry points
(sharedhashfile_amd/csrc/shf_hash_batch.hip, run_multi) and by bench.py.
"""


def shard_range(n: int, rank: int, world: int):
    """[lo, hi) of rank `rank` when n keys are split evenly over `world` ranks."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world %d/%d" % (rank, world))
    return n * rank // world, n * (rank + 1) // world


def shard_fixed(keys_flat, key_len: int, rank: int, world: int):
    """(lo, hi, view of the shard's key bytes) for a flat fixed-length key buffer."""
    n = len(keys_flat) // key_len if key_len else 0
    lo, hi = shard_range(n, rank, world)
    return lo, hi, keys_flat[lo * key_len:hi * key_len]


def shard_var(data, offsets, rank: int, world: int):
    """(lo, hi, shard bytes, rebased shard offsets) for a variable-length batch."""
    n = len(offsets) - 1
    lo, hi = shard_range(n, rank, world)
    b0, b1 = int(offsets[lo]), int(offsets[hi])
    return lo, hi, data[b0:b1], offsets[lo:hi + 1] - offsets[lo]
