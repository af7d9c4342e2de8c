#!/usr/bin/env python3
"""Round 5: the HIP runtime's pageable copies from two host threads at once --
one issuing H2D chunks, the other D2H chunks (each call holds its thread until
its copy is done) -- against one thread doing both in turn. 160 MB each way.
Then the same direction: 160 MB H2D by one thread against two threads each
copying half of it (on streams of their own).

    python tools/pageable_twothread_probe.py
"""
import ctypes
import json
import threading
import time

import numpy as np
import torch


def main():
    hip = ctypes.CDLL("libamdhip64.so", mode=ctypes.RTLD_GLOBAL)
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    n = 160 << 20
    src = np.random.default_rng(1).integers(0, 256, size=n, dtype=np.uint8)
    dst = np.empty_like(src)
    din = torch.empty(n, dtype=torch.uint8, device=dev)
    dout = torch.randint(0, 255, (n,), dtype=torch.uint8, device=dev)
    sa, sb, sc = torch.cuda.Stream(dev), torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    ha, hb, hc = ctypes.c_void_p(sa.cuda_stream), ctypes.c_void_p(sb.cuda_stream), ctypes.c_void_p(sc.cuda_stream)
    res = {}

    def h2d(chunk):
        hip.hipSetDevice(0)
        for o in range(0, n, chunk):
            assert hip.hipMemcpyAsync(ctypes.c_void_p(din.data_ptr() + o), ctypes.c_void_p(src.ctypes.data + o),
                                      ctypes.c_size_t(min(chunk, n - o)), 1, ha) == 0
        hip.hipStreamSynchronize(ha)

    def d2h(chunk):
        hip.hipSetDevice(0)
        for o in range(0, n, chunk):
            assert hip.hipMemcpyAsync(ctypes.c_void_p(dst.ctypes.data + o), ctypes.c_void_p(dout.data_ptr() + o),
                                      ctypes.c_size_t(min(chunk, n - o)), 2, hb) == 0
        hip.hipStreamSynchronize(hb)

    def h2d_part(chunk, lo, hi, st):
        hip.hipSetDevice(0)
        for o in range(lo, hi, chunk):
            assert hip.hipMemcpyAsync(ctypes.c_void_p(din.data_ptr() + o), ctypes.c_void_p(src.ctypes.data + o),
                                      ctypes.c_size_t(min(chunk, hi - o)), 1, st) == 0
        hip.hipStreamSynchronize(st)

    for chunk_mb in (4, 8, 16, 32):
        c = chunk_mb << 20
        one, two = [], []
        for _ in range(4):
            t0 = time.perf_counter()
            h2d(c)
            d2h(c)
            one.append(2 * n / (time.perf_counter() - t0) / 1e9)
            ta, tb = threading.Thread(target=h2d, args=(c,)), threading.Thread(target=d2h, args=(c,))
            t0 = time.perf_counter()
            ta.start()
            tb.start()
            ta.join()
            tb.join()
            two.append(2 * n / (time.perf_counter() - t0) / 1e9)
        same1, same2 = [], []
        for _ in range(4):
            t0 = time.perf_counter()
            h2d_part(c, 0, n, ha)
            same1.append(n / (time.perf_counter() - t0) / 1e9)
            ta = threading.Thread(target=h2d_part, args=(c, 0, n // 2, ha))
            tc = threading.Thread(target=h2d_part, args=(c, n // 2, n, hc))
            t0 = time.perf_counter()
            ta.start()
            tc.start()
            ta.join()
            tc.join()
            same2.append(n / (time.perf_counter() - t0) / 1e9)
        res["%dMiB" % chunk_mb] = {"one_thread_GB_s": [round(x, 1) for x in one[1:]],
                                   "two_threads_GB_s": [round(x, 1) for x in two[1:]],
                                   "h2d_one_thread_GB_s": [round(x, 1) for x in same1[1:]],
                                   "h2d_two_threads_GB_s": [round(x, 1) for x in same2[1:]]}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
