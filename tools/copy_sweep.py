#!/usr/bin/env python3
"""Interleaved timing of the copy-ceiling variants (include/shf_hash_batch_ceiling.h)
on fixed16's shape: 4 rotating batches of 10M x 16 B keys + 16-B outputs, plus
torch's device-to-device copy_ of the same buffers and the hash kernel itself.

    python tools/copy_sweep.py [--n 10000000] [--rounds 8] [--steps 50]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=10_000_000)
    p.add_argument("--rounds", type=int, default=8)
    p.add_argument("--steps", type=int, default=50)
    a = p.parse_args()
    import torch

    import sharedhashfile_amd as hb
    from sharedhashfile_amd.keygen import device_random_bytes

    dev = torch.device("cuda:0")
    from sharedhashfile_amd import bench_ceiling

    lib = hb.load()
    blib = bench_ceiling.load()
    n = a.n
    pairs = [(device_random_bytes(16 * n, 100 + b, dev), torch.empty((n, 2), dtype=torch.int64, device=dev))
             for b in range(4)]
    st = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    variants = {}
    for name, kind in (("copy_nt_ld", 0), ("copy4", 6), ("copy_plain", 7), ("copy_nt_ldst", 8), ("copy_sleep", 9),
                       ("copy2", 10)):
        variants[name] = (lambda kind: lambda k, o: blib.shf_hb_ceiling_async(kind, k.data_ptr(), 16 * n, None,
                                                                              o.data_ptr(), n, st()))(kind)
    variants["torch_copy_"] = lambda k, o: (o.view(torch.uint8).view(-1).copy_(k), 0)[1]
    variants["hash_k_fixed16"] = lambda k, o: lib.shf_hash_batch_fixed_kernel_async(k.data_ptr(), 16, n, 12345,
                                                                                      o.data_ptr(), 1, st())
    for f in variants.values():  # warm up
        for _ in range(20):
            for k, o in pairs:
                assert f(k, o) == 0
    torch.cuda.synchronize()
    times = {v: [] for v in variants}
    for _ in range(a.rounds):
        for v, f in variants.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for i in range(a.steps):
                k, o = pairs[i % 4]
                f(k, o)
            e1.record()
            e1.synchronize()
            times[v].append(e0.elapsed_time(e1) / a.steps)
    for v, ts in times.items():
        ts = sorted(ts)
        med = ts[len(ts) // 2]
        print("%-16s median %7.2f us  min %7.2f us  %7.1f GB/s (32 B per 16-B unit)" % (v, med * 1e3, ts[0] * 1e3,
                                                                                       n * 32 / med / 1e6))


if __name__ == "__main__":
    main()
