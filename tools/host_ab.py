#!/usr/bin/env python3
"""Interleaved A/B of library builds on the host-memory paths, in one process
(each variant its own pools and copy threads): 10M x 16-B pageable keys (one
thread, and 16 threads one slice each), 10M x U[8,512] B pageable keys.

    python tools/host_ab.py --variant head= --variant r5=@tools/_ab/lib_c4c03ae.so [--rounds 4]
"""
import argparse
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--variant", action="append", required=True)
    p.add_argument("--rounds", type=int, default=4)
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--n", type=int, default=10_000_000)
    a = p.parse_args()
    import torch

    import sharedhashfile_amd as hb
    from sharedhashfile_amd.keygen import device_random_bytes

    hb.load()
    libs = {}
    for v in a.variant:
        name, _, path = v.partition("=")
        path = os.path.join(ROOT, path[1:]) if path.startswith("@") else hb.LIB_PATH
        lib = ctypes.CDLL(path, mode=os.RTLD_LOCAL)
        for f in ("shf_hash_batch_fixed", "shf_hash_batch_var"):
            getattr(lib, f).argtypes = hb._SIGS[f]
            getattr(lib, f).restype = ctypes.c_int
        libs[name] = lib
    dev = torch.device("cuda:0")
    n = a.n
    keys = device_random_bytes(n * 16, 77, dev).cpu().numpy()
    out = np.empty((n, 2), dtype=np.uint64)
    g = torch.Generator(device=dev)
    g.manual_seed(78)
    lens = torch.randint(8, 513, (n,), generator=g, device=dev, dtype=torch.int64)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens.cpu().numpy())
    data = device_random_bytes(int(off[-1]), 79, dev).cpu().numpy()
    vout = np.empty((n, 2), dtype=np.uint64)

    def x16(lib):
        rcs = [0] * 16
        ts = [threading.Thread(target=lambda i=i: rcs.__setitem__(i, lib.shf_hash_batch_fixed(
            keys.ctypes.data + n * i // 16 * 16, 16, n * (i + 1) // 16 - n * i // 16, 12345,
            out.ctypes.data + n * i // 16 * 16, 1))) for i in range(16)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        return next((r for r in rcs if r), 0)

    cases = {"fixed16_pageable": lambda lib: lib.shf_hash_batch_fixed(keys.ctypes.data, 16, n, 12345,
                                                                       out.ctypes.data, 1),
             "fixed16_pageable_x16": x16,
             "var_pageable": lambda lib: lib.shf_hash_batch_var(data.ctypes.data, off.ctypes.data, n, 12345,
                                                                vout.ctypes.data, 1)}
    res = {}
    for r in range(a.rounds):
        for case, fn in cases.items():
            for name, lib in libs.items():
                for _ in range(2):
                    assert fn(lib) == 0
                for _ in range(a.reps):
                    t0 = time.perf_counter()
                    assert fn(lib) == 0
                    res.setdefault("%s/%s" % (case, name), []).append(n / (time.perf_counter() - t0) / 1e9)
        print("round %d" % r, file=sys.stderr, flush=True)
    print(json.dumps({k: {"median": round(float(np.median(v)), 3), "min": round(min(v), 3),
                          "max": round(max(v), 3)} for k, v in sorted(res.items())}))


if __name__ == "__main__":
    main()
