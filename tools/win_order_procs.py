#!/usr/bin/env python3
"""The window order's use on the host, measured: the reference's own put and
get loops (oracle/_ref/libref_shf.so, one store, T forked worker processes each
with its own handle: the reference's multi-process use) over n 16-B keys,
  batch order:  worker t takes keys [t n / T, (t+1) n / T) of the batch;
  window order: worker t takes windows [256 t / T, 256 (t+1) / T) of the GPU's
                window order (shf_win_order's perm and win_start), so no two
                workers share a window's lock or structures.
The GPU part (hashes + order, through the library) runs in this process; the
workers are forked by a child python that never touches the GPU.

    python tools/win_order_procs.py OUT.json [n] [T ...]
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CHILD = r'''
import json, sys, tempfile
import numpy as np
sys.path.insert(0, %r)
from oracle.oracle_py import reference_put_get_procs
z = np.load(%r)
data, off, h, perm, ws = z["data"], z["off"], z["h"], z["perm"], z["ws"]
n = off.size - 1
out = []
for T in %r:
    even = np.array([n * t // T for t in range(T + 1)], np.uint64)
    wst = np.array([ws[256 * t // T] for t in range(T + 1)], np.uint64)
    for rep in range(2):
        for name, order, st in (("batch", None, even), ("window", perm, wst)):
            with tempfile.TemporaryDirectory(dir="/dev/shm") as d:
                f, ps, gs = reference_put_get_procs(data, off, h, order, st, d, "s", 1)
            r = {"procs": T, "order": name, "rep": rep, "found": int(f), "put_ns_per_key": ps / n * 1e9,
                 "get_ns_per_key": gs / n * 1e9}
            print(json.dumps(r), flush=True)
            out.append(r)
print("RESULT " + json.dumps(out), flush=True)
'''


def main():
    import sharedhashfile_amd as hb

    out = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4_000_000
    procs = [int(x) for x in sys.argv[3:]] or [4, 16]
    rng = np.random.default_rng(7)
    k = rng.integers(0, 256, size=(n, 16), dtype=np.uint8)
    k[:, :8] = np.arange(n, dtype="<u8").view(np.uint8).reshape(n, 8)  # distinct keys
    data = k.reshape(-1)
    off = np.arange(n + 1, dtype=np.uint64) * 16
    h = hb.hash_var_host(data, off)
    perm, ws = hb.win_order_host(h)
    with tempfile.NamedTemporaryFile(dir="/dev/shm", suffix=".npz", delete=False) as f:
        path = f.name
    try:
        np.savez(path, data=data, off=off, h=h, perm=perm, ws=ws)
        p = subprocess.run([sys.executable, "-u", "-c", CHILD % (ROOT, path, procs)], capture_output=True, text=True,
                           timeout=1200)
    finally:
        os.unlink(path)
    sys.stdout.write(p.stdout)
    sys.stderr.write(p.stderr[-3000:])
    rows = json.loads([l for l in p.stdout.splitlines() if l.startswith("RESULT ")][-1][7:])
    summary = []
    for T in procs:
        med = lambda o, key: float(np.median([r[key] for r in rows if r["procs"] == T and r["order"] == o]))
        summary.append({"procs": T, "n": n, "put_speedup": med("batch", "put_ns_per_key") / med("window", "put_ns_per_key"),
                        "get_speedup": med("batch", "get_ns_per_key") / med("window", "get_ns_per_key"),
                        "all_found": all(r["found"] == n for r in rows if r["procs"] == T)})
        print(json.dumps(summary[-1]), flush=True)
    with open(out, "w") as f:
        json.dump({"summary": summary, "runs": rows}, f, indent=1)


if __name__ == "__main__":
    main()
