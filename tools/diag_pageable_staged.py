#!/usr/bin/env python3
"""Where the pageable staged host path's spread comes from.

Times shf_hash_batch_fixed(MEM_HOST) over pageable numpy buffers (the staged
pipeline, the only path for pageable memory since round 5 -- chunked par_memcpy into
pinned staging, H2D, kernel, direct stores into pinned staging, drain copy),
--repeats times, and records per repeat: wall time, minor page faults,
voluntary / involuntary context switches, process CPU time, and the cgroup's
CFS throttling (cpu.stat nr_throttled / throttled_usec) -- so a slow repeat can
be attributed to first-touch faults, the copy threads being descheduled, or
the cgroup's CPU quota.

    python tools/diag_pageable_staged.py [--n 10000000] [--repeats 20] [--fresh-out]
"""
import argparse
import json
import os
import resource
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def cgroup_cpu_stat():
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            return {k: int(v) for k, v in (line.split() for line in f if line.strip())}
    except OSError:
        return {}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=10_000_000)
    p.add_argument("--repeats", type=int, default=20)
    p.add_argument("--fresh-out", action="store_true", help="a new (never touched) output array every repeat")
    p.add_argument("--env", action="append", default=[], help="NAME=VALUE set before the calls")
    p.add_argument("--trace-file", default=None, help="where this run's stderr goes (with SHF_HB_TRACE=1)")
    a = p.parse_args()
    for kv in a.env:
        k, _, v = kv.partition("=")
        os.environ[k] = v
    import sharedhashfile_amd as hb
    from sharedhashfile_amd.keygen import splitmix_bytes

    lib = hb.load()
    keys = np.frombuffer(splitmix_bytes(a.n * 16, 77), dtype=np.uint8).copy()
    out = np.empty((a.n, 2), dtype=np.uint64)
    assert lib.shf_hash_batch_fixed(keys.ctypes.data, 16, a.n, 12345, out.ctypes.data, hb.MEM_HOST) == 0
    rows = []
    for r in range(a.repeats):
        o = np.empty((a.n, 2), dtype=np.uint64) if a.fresh_out else out
        c0, u0 = cgroup_cpu_stat(), resource.getrusage(resource.RUSAGE_SELF)
        t0 = time.perf_counter()
        rc = lib.shf_hash_batch_fixed(keys.ctypes.data, 16, a.n, 12345, o.ctypes.data, hb.MEM_HOST)
        dt = time.perf_counter() - t0
        c1, u1 = cgroup_cpu_stat(), resource.getrusage(resource.RUSAGE_SELF)
        assert rc == 0
        rows.append({"repeat": r, "ms": round(dt * 1e3, 3), "gkeys_s": round(a.n / dt / 1e9, 3),
                     "minflt": u1.ru_minflt - u0.ru_minflt, "majflt": u1.ru_majflt - u0.ru_majflt,
                     "nvcsw": u1.ru_nvcsw - u0.ru_nvcsw, "nivcsw": u1.ru_nivcsw - u0.ru_nivcsw,
                     "cpu_ms": round((u1.ru_utime + u1.ru_stime - u0.ru_utime - u0.ru_stime) * 1e3, 2),
                     "cg_throttled": c1.get("nr_throttled", 0) - c0.get("nr_throttled", 0),
                     "cg_throttled_ms": round((c1.get("throttled_usec", 0) - c0.get("throttled_usec", 0)) / 1e3, 2)})
    v = np.array([x["gkeys_s"] for x in rows])
    # SHF_HB_TRACE=1: the library's own per-call split (stderr lines, in call order)
    if os.environ.get("SHF_HB_TRACE") == "1" and a.trace_file and os.path.exists(a.trace_file):
        tr = [l for l in open(a.trace_file) if l.startswith("shf_hash_batch trace:")][-a.repeats:]
        for row, line in zip(rows, tr):
            row.update({kv.split("=")[0]: float(kv.split("=")[1]) for kv in line.split()[2:]
                        if kv.split("=")[0].endswith("_ms")})
    summary = {"n": a.n, "fresh_out": a.fresh_out, "env": a.env, "median": float(np.median(v)), "min": float(v.min()),
               "max": float(v.max()), "spread_max_over_min": round(float(v.max() / v.min()), 3),
               "cgroup_cpu_max": open("/sys/fs/cgroup/cpu.max").read().strip() if os.path.exists(
                   "/sys/fs/cgroup/cpu.max") else None, "cpus_affinity": len(os.sched_getaffinity(0))}
    print(json.dumps({"summary": summary, "repeats": rows}))


if __name__ == "__main__":
    main()
