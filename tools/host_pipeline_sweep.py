#!/usr/bin/env python3
"""Host-memory pipeline shape sweep for the SHF_HASH_MEM_HOST calls:
SHF_HB_STAGE_MB (MiB of key bytes per chunk) x SHF_HB_SLOTS (chunks in flight),
keys/s for 10M x 16 B keys (configs[1]) from pageable and from page-locked
buffers, and 2M x U[8,512] B variable-length keys from pageable buffers. Every
shape must give the same hashes. The library reads both knobs on every call.

    python tools/host_pipeline_sweep.py > profiles/r1/host_pipeline_sweep.txt
"""
import hashlib
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import sharedhashfile_amd as hb
    from sharedhashfile_amd.keygen import splitmix_bytes, splitmix_lengths

    lib = hb.load()
    n = 10_000_000
    keys = np.frombuffer(splitmix_bytes(n * 16, 77), dtype=np.uint8).copy()
    out = np.empty((n, 2), dtype=np.uint64)
    pk = torch.from_numpy(keys).pin_memory()
    po = torch.empty((n, 2), dtype=torch.int64).pin_memory()
    m = 2_000_000
    off = np.zeros(m + 1, dtype=np.uint64)
    off[1:] = np.cumsum(splitmix_lengths(m, 8, 512, 5))
    data = np.frombuffer(splitmix_bytes(int(off[-1]), 6), dtype=np.uint8).copy()
    vout = np.empty((m, 2), dtype=np.uint64)

    cases = [
        ("fixed16", "pageable", n,
         lambda: lib.shf_hash_batch_fixed(keys.ctypes.data, 16, n, 12345, out.ctypes.data, hb.MEM_HOST), lambda: out),
        ("fixed16", "pinned", n,
         lambda: lib.shf_hash_batch_fixed(pk.data_ptr(), 16, n, 12345, po.data_ptr(), hb.MEM_HOST), lambda: po.numpy()),
        ("var", "pageable", m,
         lambda: lib.shf_hash_batch_var(data.ctypes.data, off.ctypes.data, m, 12345, vout.ctypes.data, hb.MEM_HOST),
         lambda: vout),
    ]
    digests = {}
    print("G keys/s, host buffers in and out (%d x 16 B keys; %d x U[8,512] B keys, %.0f MB)" % (n, m, off[-1] / 1e6))
    print("%8s %5s %18s %18s %18s" % ("stage_MB", "slots", "16B pageable", "16B pinned", "var pageable"))
    shapes = [(mb, slots, 8) for mb in (4, 8, 16, 32, 64) for slots in (2, 3, 4)]
    if len(sys.argv) > 1 and sys.argv[1] == "--threads":  # staging-copy threads at the default shape
        shapes = [(32, 3, t) for t in (2, 4, 8, 12, 16, 24)]
        print("(rows: SHF_HB_COPY_THREADS = 2, 4, 8, 12, 16, 24 at 32 MiB x 3 slots)")
    for mb, slots, threads in shapes:
            os.environ["SHF_HB_STAGE_MB"] = str(mb)
            os.environ["SHF_HB_SLOTS"] = str(slots)
            os.environ["SHF_HB_COPY_THREADS"] = str(threads)
            row = []
            for kind, mem, count, fn, res in cases:
                rc = fn()  # warm: staging buffers for this shape
                if rc:
                    raise hb.ShfHashBatchError(rc, kind)
                reps = 5
                t0 = time.perf_counter()
                for _ in range(reps):
                    rc = fn()
                    if rc:
                        raise hb.ShfHashBatchError(rc, kind)
                dt = (time.perf_counter() - t0) / reps
                d = hashlib.sha256(np.ascontiguousarray(res()).tobytes()).hexdigest()
                assert digests.setdefault(kind, d) == d, (kind, mem, mb, slots)
                row.append("%18.3f" % (count / dt / 1e9))
            print("%8d %5d %s  threads=%d" % (mb, slots, " ".join(row), threads), flush=True)
    print("hashes identical across shapes:", {k: v[:16] for k, v in digests.items()})


if __name__ == "__main__":
    main()
