#!/usr/bin/env python3
"""Config D's hash-phase balance: for U[8,512]-byte keys in
64-key tiles, how many block-steps a tile's wave runs (its longest key) against
the work its lanes do (the mean), and what length-sorting the 128 keys of two
tiles into a long and a short wave would give. A block-step = one 16-B body
block; +1 for the tail / finalisation."""
import numpy as np


def main(tiles=200_000, lo=8, hi=512, seed=1):
    rng = np.random.default_rng(seed)
    nb = (rng.integers(lo, hi + 1, size=64 * tiles) >> 4) + 1
    t = nb.reshape(-1, 64)
    mx, mean = t.max(1).mean(), t.mean()
    p = np.sort(nb.reshape(-1, 128), axis=1)
    short, long_ = p[:, :64].max(1).mean(), p[:, 64:].max(1).mean()
    print("tile: mean %.2f block-steps, longest %.2f -> lane efficiency %.3f" % (mean, mx, mean / mx))
    print("two tiles length-sorted: waves' longest %.2f and %.2f -> %.3f" % (long_, short, mean / ((long_ + short) / 2)))


if __name__ == "__main__":
    main()
