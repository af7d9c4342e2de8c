#!/usr/bin/env python3
"""Host-memory UID parts vs 16-B hashes: keys/s of
shf_uid_parts_batch_fixed / shf_hash_batch_fixed on 10M pageable (and
page-locked) 16-B keys, per pipeline setting, alternating the settings round by
round so box drift spreads evenly; with SHF_HB_TRACE=1 the library's own
per-call split (staging in / enqueue / waits / copy-out) is kept per repeat.

    python tools/host_uid_sweep.py [--n 10000000] [--rounds 3] [--reps 5]
        [--set NAME:ENV=V,ENV=V ...] > gpurun_out/host_uid_sweep.json
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

DEFAULT_SETS = ["default:", "stage8:SHF_HB_STAGE_MB=8", "stage32:SHF_HB_STAGE_MB=32,SHF_HB_POOL_MB=128",
                "stage64:SHF_HB_STAGE_MB=64,SHF_HB_POOL_MB=256", "slots2:SHF_HB_SLOTS=2",
                "copy4:SHF_HB_COPY_THREADS=4", "cpu_h2d:SHF_HB_RUNTIME_H2D=0"]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=10_000_000)
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--reps", type=int, default=5)
    p.add_argument("--set", action="append", default=None)
    p.add_argument("--modes", default="uid,hash,uid_pinned_staged,hash_pinned_staged")
    a = p.parse_args()
    import torch

    import sharedhashfile_amd as hb
    from sharedhashfile_amd.keygen import splitmix_bytes

    lib = hb.load()
    n = a.n
    keys = np.frombuffer(splitmix_bytes(n * 16, 77), dtype=np.uint8).copy()
    parts = np.empty(n, dtype=np.uint64)
    hashes = np.empty((n, 2), dtype=np.uint64)
    pk = torch.from_numpy(keys).pin_memory()
    pparts = torch.empty(n, dtype=torch.int64).pin_memory()
    phash = torch.empty((n, 2), dtype=torch.int64).pin_memory()
    calls = {
        "uid": lambda: lib.shf_uid_parts_batch_fixed(keys.ctypes.data, 16, n, 12345, parts.ctypes.data, hb.MEM_HOST),
        "hash": lambda: lib.shf_hash_batch_fixed(keys.ctypes.data, 16, n, 12345, hashes.ctypes.data, hb.MEM_HOST),
        "uid_pinned": lambda: lib.shf_uid_parts_batch_fixed(pk.data_ptr(), 16, n, 12345, pparts.data_ptr(),
                                                            hb.MEM_HOST),
        "uid_pinned_staged": lambda: lib.shf_uid_parts_batch_fixed(pk.data_ptr(), 16, n, 12345, pparts.data_ptr(),
                                                                   hb.MEM_HOST),
        "hash_pinned_staged": lambda: lib.shf_hash_batch_fixed(pk.data_ptr(), 16, n, 12345, phash.data_ptr(),
                                                               hb.MEM_HOST),
    }
    sets = []
    for spec in a.set or DEFAULT_SETS:
        name, _, envs = spec.partition(":")
        sets.append((name, dict(kv.split("=", 1) for kv in envs.split(",") if kv)))
    base = dict(os.environ)
    res = {}
    for r in range(a.rounds):
        for name, env in sets:
            for mode in a.modes.split(","):
                os.environ.clear()
                os.environ.update(base)
                os.environ.update(env)
                if mode.endswith("pinned_staged"):
                    os.environ["SHF_HB_ZERO_COPY_MAX_KEY"] = "0"
                fn = calls[mode]
                assert fn() == 0
                ts = []
                for _ in range(a.reps):
                    t0 = time.perf_counter()
                    rc = fn()
                    ts.append(time.perf_counter() - t0)
                    assert rc == 0
                res.setdefault("%s/%s" % (name, mode), []).extend(n / t / 1e9 for t in ts)
        print("round %d done" % r, file=sys.stderr, flush=True)
    os.environ.clear()
    os.environ.update(base)
    out = {k: {"median": round(float(np.median(v)), 3), "min": round(min(v), 3), "max": round(max(v), 3)}
           for k, v in res.items()}
    print(json.dumps({"n": n, "rounds": a.rounds, "reps": a.reps, "gkeys_s": out}))


if __name__ == "__main__":
    main()
