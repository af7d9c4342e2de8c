#!/usr/bin/env python3
"""Round 5: how fast the HIP runtime's own pageable copies are (hipMemcpyAsync
with a pageable host pointer: the runtime stages or pins the pages itself),
against a page-locked buffer's copies and against host memcpy, for 160 MB in
chunks of 4-32 MiB -- to decide whether the staged pipeline should hand the
caller's pageable keys to the runtime instead of copying them into its pinned
slots on the CPU first.

    python tools/pageable_dma_probe.py
"""
import ctypes
import json
import time

import numpy as np
import torch


def main():
    hip = ctypes.CDLL("libamdhip64.so", mode=ctypes.RTLD_GLOBAL)
    dev = torch.device("cuda:0")
    n = 160 << 20
    src = np.random.default_rng(1).integers(0, 256, size=n, dtype=np.uint8)
    dst = np.empty_like(src)
    pinned = torch.empty(n, dtype=torch.uint8).pin_memory()
    d = torch.empty(n, dtype=torch.uint8, device=dev)
    st = torch.cuda.Stream(dev)
    h = ctypes.c_void_p(st.cuda_stream)
    res = {}

    def timeit(fn, reps=5):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return round(n / min(ts) / 1e9, 2), round(n / float(np.median(ts)) / 1e9, 2)

    for chunk_mb in (4, 8, 16, 32, 160):
        c = chunk_mb << 20

        def h2d(ptr):
            for o in range(0, n, c):
                hip.hipMemcpyAsync(ctypes.c_void_p(d.data_ptr() + o), ctypes.c_void_p(ptr + o), ctypes.c_size_t(min(c, n - o)),
                                   1, h)
            hip.hipStreamSynchronize(h)

        def d2h(ptr):
            for o in range(0, n, c):
                hip.hipMemcpyAsync(ctypes.c_void_p(ptr + o), ctypes.c_void_p(d.data_ptr() + o), ctypes.c_size_t(min(c, n - o)),
                                   2, h)
            hip.hipStreamSynchronize(h)

        res["h2d_pageable_%dMiB" % chunk_mb] = timeit(lambda: h2d(src.ctypes.data))
        res["d2h_pageable_%dMiB" % chunk_mb] = timeit(lambda: d2h(dst.ctypes.data))
        res["h2d_pinned_%dMiB" % chunk_mb] = timeit(lambda: h2d(pinned.data_ptr()))
        res["d2h_pinned_%dMiB" % chunk_mb] = timeit(lambda: d2h(pinned.data_ptr()))
    res["host_memcpy_1thread"] = timeit(lambda: np.copyto(dst, src))
    print(json.dumps({"GB_per_s_best_median": res}))


if __name__ == "__main__":
    main()
