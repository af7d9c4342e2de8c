#!/usr/bin/env python3
"""f4's read traffic model: records of the synthetic tabs
(sharedhashfile_amd/tabgen.py: 9-B header + key U[16,64] + value U[8,128])
packed back to back after the 65 560-B rows; each record read on its own
touches ceil((start % 128 + len) / 128) 128-B lines. Fetched over algorithmic
bytes when no line is shared between two records' reads."""
import numpy as np


def main(n=1_000_000, seed=0):
    rng = np.random.default_rng(seed)
    L = 9 + rng.integers(16, 65, n) + rng.integers(8, 129, n)
    start = 65560 + np.concatenate([[0], np.cumsum(L)[:-1]])
    lines = (start % 128 + L + 127) // 128
    print("mean record %.1f B, lines per record %.3f, fetched / record bytes %.3f"
          % (L.mean(), lines.mean(), lines.mean() * 128 / L.mean()))


if __name__ == "__main__":
    main()
