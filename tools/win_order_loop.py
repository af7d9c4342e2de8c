#!/usr/bin/env python3
"""The point of the window order, measured on the box's host: the reference's
own put and get loops (oracle/_ref/libref_shf.so: shf_put_key_val /
shf_get_key_val_copy with the hashes in the thread-local seam,
test.9.shf.c:176-182) over n keys, in batch order and in the window order the
GPU computed (shf_win_order), each in a fresh store on /dev/shm, alternated.
Hashes and order come from the library (GPU); the stores are checked equal.

    python tools/win_order_loop.py OUT.json [n ...]
"""
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def keys(n, seed=7):
    rng = np.random.default_rng(seed)
    k = rng.integers(0, 256, size=(n, 16), dtype=np.uint8)
    k[:, :8] = np.arange(n, dtype="<u8").view(np.uint8).reshape(n, 8)  # distinct
    off = np.arange(n + 1, dtype=np.uint64) * 16
    return k.reshape(-1), off


def main():
    import sharedhashfile_amd as hb
    from oracle.oracle_py import reference_put_in_order, store_files

    out = sys.argv[1]
    sizes = [int(x) for x in sys.argv[2:]] or [1_000_000, 4_000_000]
    res = []
    for n in sizes:
        data, off = keys(n)
        t0 = time.time()
        h = hb.hash_var_host(data, off)
        perm, start = hb.win_order_host(h)
        t1 = time.time()
        rows = []
        for rep in range(2):
            for name, order in (("batch", None), ("window", perm)):
                with tempfile.TemporaryDirectory(dir="/dev/shm") as d:
                    found, uids, ps, gs = reference_put_in_order(data, off, h, order, d, "s", 1)
                    if rep == 0 and name == "batch":
                        ref_files = {k: hash(v) for k, v in store_files(d, "s").items()}
                        ref_uids = uids
                    elif rep == 0:
                        same = ({k: hash(v) for k, v in store_files(d, "s").items()} == ref_files and
                                bool((uids == ref_uids).all()))
                assert found == n, (name, found)
                rows.append({"order": name, "rep": rep, "put_ns_per_key": ps / n * 1e9, "get_ns_per_key": gs / n * 1e9})
                print(n, rows[-1], flush=True)
        med = lambda o, k: float(np.median([r[k] for r in rows if r["order"] == o]))
        r = {"n": n, "gpu_hash_and_order_s": t1 - t0, "store_identical": same, "runs": rows,
             "put_speedup": med("batch", "put_ns_per_key") / med("window", "put_ns_per_key"),
             "get_speedup": med("batch", "get_ns_per_key") / med("window", "get_ns_per_key")}
        print(json.dumps({k: v for k, v in r.items() if k != "runs"}), flush=True)
        res.append(r)
    with open(out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
