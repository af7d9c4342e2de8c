#!/usr/bin/env python3
"""Round 5: k threads each hashing a 1/k slice of one pageable 16-B batch at once
(bench.py's fixed16_pageable_x16 shape), repeated; aggregate G keys/s per
repeat and, with SHF_HB_TRACE=1 in the environment, the per-call stage times the
library prints (total, copy_in, enqueue, wait, copy_out) summarised.

    SHF_HB_TRACE=1 python tools/diag_threads.py --threads 16 [--n 10000000] [--repeats 5] 2> trace.err
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=10_000_000)
    p.add_argument("--threads", type=int, default=16)
    p.add_argument("--repeats", type=int, default=5)
    a = p.parse_args()
    import sharedhashfile_amd as hb

    lib = hb.load()
    keys = np.random.default_rng(1).integers(0, 256, size=a.n * 16, dtype=np.uint8)
    out = np.empty((a.n, 2), dtype=np.uint64)
    k = a.threads

    def wave():
        rcs = [0] * k

        def one(i):
            lo, hi = a.n * i // k, a.n * (i + 1) // k
            rcs[i] = lib.shf_hash_batch_fixed(keys.ctypes.data + lo * 16, 16, hi - lo, 12345,
                                              out.ctypes.data + lo * 16, hb.MEM_HOST)

        ts = [threading.Thread(target=one, args=(i,)) for i in range(k)]
        t0 = time.perf_counter()
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        dt = time.perf_counter() - t0
        assert rcs == [0] * k
        return a.n / dt / 1e9

    wave()
    rates = [wave() for _ in range(a.repeats)]
    print(json.dumps({"threads": k, "n": a.n, "gkeys_s": [round(r, 3) for r in rates],
                      "env": {e: os.environ.get(e) for e in ("SHF_HB_POOL_MB", "SHF_HB_COPY_THREADS", "SHF_HB_SLOTS",
                                                             "SHF_HB_STAGE_MB")}}))


if __name__ == "__main__":
    main()
