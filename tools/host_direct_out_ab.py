#!/usr/bin/env python3
"""Host-inclusive A/B of SHF_HB_DIRECT_OUT (staged pipelines whose kernel
stores the hashes into the page-locked output, or the slot's page-locked
staging for a pageable output, vs a D2H copy per chunk),
interleaved in one process; outputs of both modes compared.

    python tools/host_direct_out_ab.py [--n 10000000] [--reps 5]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=10_000_000)
    p.add_argument("--reps", type=int, default=5)
    a = p.parse_args()
    import torch

    import sharedhashfile_amd as hb
    from sharedhashfile_amd.keygen import device_random_bytes

    dev = torch.device("cuda", 0)
    lib = hb.load()
    n = a.n
    seed = 12345
    k16 = torch.from_numpy(device_random_bytes(n * 16, 77, dev).cpu().numpy()).pin_memory()
    n256 = n // 8
    k256 = torch.from_numpy(device_random_bytes(n256 * 256, 78, dev).cpu().numpy()).pin_memory()
    g = torch.Generator(device=dev)
    g.manual_seed(79)
    lens = torch.randint(8, 513, (n,), generator=g, device=dev, dtype=torch.int64).cpu().numpy()
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    data = torch.from_numpy(device_random_bytes(int(off[-1]), 80, dev).cpu().numpy()).pin_memory()
    poff = torch.from_numpy(off.view(np.int64)).pin_memory()
    outs = {m: {c: torch.empty((nn, 2), dtype=torch.int64).pin_memory() for c, nn in
                (("fixed16_staged", n), ("fixed256", n256), ("var", n))} for m in "01"}
    k16p = k16.numpy()
    outp = {m: np.empty((n, 2), dtype=np.uint64) for m in "01"}
    cases = {
        "fixed16_pageable": (n, lambda o: lib.shf_hash_batch_fixed(k16p.ctypes.data, 16, n, seed, o.ctypes.data,
                                                                   hb.MEM_HOST)),
        "fixed16_staged": (n, lambda o: lib.shf_hash_batch_fixed(k16.data_ptr(), 16, n, seed, o.data_ptr(), hb.MEM_HOST)),
        "fixed256": (n256, lambda o: lib.shf_hash_batch_fixed(k256.data_ptr(), 256, n256, seed, o.data_ptr(),
                                                              hb.MEM_HOST)),
        "var": (n, lambda o: lib.shf_hash_batch_var(data.data_ptr(), poff.data_ptr(), n, seed, o.data_ptr(),
                                                   hb.MEM_HOST)),
    }
    os.environ["SHF_HB_ZERO_COPY_MAX_KEY"] = "0"  # 16-B keys through the staged pipeline
    ts = {(c, m): [] for c in cases for m in "01"}
    for r in range(a.reps + 1):
        for c, (nn, fn) in cases.items():
            for m in "01":
                os.environ["SHF_HB_DIRECT_OUT"] = m
                t0 = time.perf_counter()
                rc = fn(outp[m] if c == "fixed16_pageable" else outs[m][c])
                dt = time.perf_counter() - t0
                assert rc == 0, (c, m, rc)
                if r:
                    ts[(c, m)].append(dt)
    for c, (nn, _) in cases.items():
        same = (np.array_equal(outp["0"], outp["1"]) if c == "fixed16_pageable"
                else torch.equal(outs["0"][c], outs["1"][c]))
        for m in "01":
            t = float(np.median(ts[(c, m)]))
            print("%-16s direct_out=%s  median %8.2f ms  %6.3f G keys/s  outputs equal: %s" % (c, m, t * 1e3,
                                                                                             nn / t / 1e9, same))


if __name__ == "__main__":
    main()
