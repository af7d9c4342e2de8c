#!/usr/bin/env python3
"""Round 5: do the HIP runtime's pageable copies overlap? 160 MB each way in
chunks: (a) every H2D then every D2H on one stream; (b) H2D of chunk i on one
stream beside D2H of chunk i - 1 on another (what a pipeline that hands
pageable memory to the runtime would do); (c) the same with page-locked
buffers. Also how long the host thread is held inside the copy calls.

    python tools/pageable_overlap_probe.py
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
    psrc = torch.from_numpy(src.copy()).pin_memory()
    pdst = torch.empty(n, dtype=torch.uint8).pin_memory()
    din = torch.empty(n, dtype=torch.uint8, device=dev)
    dout = torch.randint(0, 255, (n,), dtype=torch.uint8, device=dev)
    sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    ha, hb = ctypes.c_void_p(sa.cuda_stream), ctypes.c_void_p(sb.cuda_stream)
    res = {}

    def cp(dptr, sptr, size, kind, h):
        rc = hip.hipMemcpyAsync(ctypes.c_void_p(dptr), ctypes.c_void_p(sptr), ctypes.c_size_t(size), kind, h)
        assert rc == 0, rc

    def run(chunk, h_src, h_dst, overlap):
        issue = 0.0
        t0 = time.perf_counter()
        for i, o in enumerate(range(0, n, chunk)):
            c = min(chunk, n - o)
            ti = time.perf_counter()
            cp(din.data_ptr() + o, h_src + o, c, 1, ha)
            if overlap and o:
                cp(h_dst + o - chunk, dout.data_ptr() + o - chunk, chunk, 2, hb)
            issue += time.perf_counter() - ti
        if overlap:
            cp(h_dst + (n - chunk), dout.data_ptr() + (n - chunk), chunk, 2, hb)
        else:
            hip.hipStreamSynchronize(ha)
            for o in range(0, n, chunk):
                cp(h_dst + o, dout.data_ptr() + o, min(chunk, n - o), 2, ha)
        hip.hipStreamSynchronize(ha)
        hip.hipStreamSynchronize(hb)
        dt = time.perf_counter() - t0
        return round(2 * n / dt / 1e9, 1), round(issue * 1e3, 2)

    for chunk_mb in (8, 16):
        c = chunk_mb << 20
        for name, s_, d_ in (("pageable", src.ctypes.data, dst.ctypes.data), ("pinned", psrc.data_ptr(), pdst.data_ptr())):
            for ov in (False, True):
                run(c, s_, d_, ov)
                r = [run(c, s_, d_, ov) for _ in range(3)]
                res["%s_%dMiB_%s" % (name, chunk_mb, "overlap" if ov else "sequential")] = {
                    "GB_s_both_directions": [x[0] for x in r], "host_ms_in_calls": [x[1] for x in r]}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
