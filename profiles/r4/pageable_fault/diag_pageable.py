#!/usr/bin/env python3
"""Diagnostic: pageable zero-copy path (SHF_HB_PAGEABLE_ZERO_COPY) on a few buffer kinds."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sharedhashfile_amd as hb  # noqa: E402
from oracle.oracle_py import Oracle  # noqa: E402
from sharedhashfile_amd.keygen import splitmix_bytes  # noqa: E402

lib = hb.load()
o = Oracle()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 5_000_000
for kind in ("bytes", "numpy"):
    raw = splitmix_bytes(n * 16, 21)
    flat = np.frombuffer(raw, dtype=np.uint8) if kind == "bytes" else np.frombuffer(raw, dtype=np.uint8).copy()
    want = o.hash_fixed(flat, 16, threads=8)
    for env in ("0", "1"):
        os.environ["SHF_HB_PAGEABLE_ZERO_COPY"] = env
        out = np.zeros((n, 2), dtype=np.uint64)
        rc = lib.shf_hash_batch_fixed(flat.ctypes.data, 16, n, 12345, out.ctypes.data, hb.MEM_HOST)
        print(kind, "zc=" + env, "rc", rc, "hip", lib.shf_hash_batch_last_hip_error(), "ok",
              bool(np.array_equal(out, want)), "keys@%x out@%x" % (flat.ctypes.data, out.ctypes.data), flush=True)
