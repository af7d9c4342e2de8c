#!/usr/bin/env python3
"""*_multi host batches split into 1/2/4/8 shards that share this one GPU
(SHF_HB_MULTI_SHARE_DEVICES=1), from pageable buffers: what an 8-GPU host
caller's shard threads do to the shared copy workers and staging pools
(VERDICT r5 item 4 / weak 8). Keys/s per (shards, pool MiB, copy threads),
alternating settings round by round.

    python tools/multi_share_sweep.py [--n 100000000] [--rounds 2] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=100_000_000)
    p.add_argument("--rounds", type=int, default=2)
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--shards", default="1,2,4,8")
    p.add_argument("--pools", default="64,512")
    p.add_argument("--copy-threads", default="12")
    p.add_argument("--var-n", type=int, default=10_000_000)
    a = p.parse_args()
    import torch

    import sharedhashfile_amd as hb
    from sharedhashfile_amd.keygen import device_random_bytes

    lib = hb.load()
    dev = torch.device("cuda:0")
    n = a.n
    keys = device_random_bytes(n * 16, 5, dev).cpu().numpy()
    out = np.empty((n, 2), dtype=np.uint64)
    m = a.var_n
    g = torch.Generator(device=dev)
    g.manual_seed(6)
    lens = torch.randint(8, 513, (m,), generator=g, device=dev, dtype=torch.int64)
    off = np.zeros(m + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens.cpu().numpy())
    data = device_random_bytes(int(off[-1]), 7, dev).cpu().numpy()
    vout = np.empty((m, 2), dtype=np.uint64)
    os.environ["SHF_HB_MULTI_SHARE_DEVICES"] = "1"
    res = {}
    for r in range(a.rounds):
        for pool in a.pools.split(","):
            for ct in a.copy_threads.split(","):
                os.environ["SHF_HB_POOL_MB"] = pool
                os.environ["SHF_HB_COPY_THREADS"] = ct
                for s in (int(x) for x in a.shards.split(",")):
                    for kind in ("fixed16", "var"):
                        if kind == "fixed16":
                            fn = lambda: lib.shf_hash_batch_fixed_multi(keys.ctypes.data, 16, n, 12345,  # noqa: E731
                                                                        out.ctypes.data, s)
                            cnt = n
                        else:
                            fn = lambda: lib.shf_hash_batch_var_multi(data.ctypes.data, off.ctypes.data, m,  # noqa: E731
                                                                      12345, vout.ctypes.data, s)
                            cnt = m
                        assert fn() == 0
                        for _ in range(a.reps):
                            t0 = time.perf_counter()
                            assert fn() == 0
                            res.setdefault("%s/shards%d/pool%s/ct%s" % (kind, s, pool, ct), []).append(
                                cnt / (time.perf_counter() - t0) / 1e9)
                        lib.shf_hash_batch_release()
        print("round %d done" % r, file=sys.stderr, flush=True)
    print(json.dumps({"n": n, "var_n": m, "gkeys_s": {k: {"median": round(float(np.median(v)), 3),
                                                          "min": round(min(v), 3), "max": round(max(v), 3)}
                                                      for k, v in res.items()}}))


if __name__ == "__main__":
    main()
