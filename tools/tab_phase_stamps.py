#!/usr/bin/env python3
"""Phase timing of the f4 tab copy from in-kernel stamps (a -DSHFHB_TAB_STAMPS=1
build of the library): the bench's tab-part batch, one launch, then per
workgroup the 100-MHz real-time stamps at kernel start, after each segment's
scan barrier (refs + length words read, scanned), after its row barrier (rows
written, record lists built), after its chunk copy, after the last partial
chunks and at the end.

    python tools/tab_phase_stamps.py build/ab/lib_stamps.so [--n 1024]
"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("lib")
    p.add_argument("--n", type=int, default=1024)
    a = p.parse_args()
    import torch

    import bench
    import sharedhashfile_amd as hb

    dev = torch.device("cuda", 0)
    lib = hb.load(os.path.abspath(a.lib))
    lib.shf_tab_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint64]

    class _A:
        tab_jobs = a.n

    tw = bench.tab_workload(_A, dev, 0x5348460000000001)
    src, dst, d_jobs, d_maps, prm = tw.keep
    out = torch.zeros_like(dst)

    def call():
        rc = lib.shf_tab_copy_batch_async(ctypes.c_void_p(src.data_ptr()), src.numel(), ctypes.c_void_p(out.data_ptr()),
                                          out.numel(), ctypes.c_void_p(d_jobs.data_ptr()), a.n,
                                          ctypes.c_void_p(d_maps.data_ptr()), 8, ctypes.byref(prm), None)
        assert rc == 0, rc
        torch.cuda.synchronize()

    for _ in range(3):
        call()
    st = np.zeros(4096 * 16, dtype=np.uint64)
    assert lib.shf_tab_debug_stamps(st.ctypes.data, st.size) == 0
    s = st.reshape(4096, 16)[:a.n].astype(np.int64)
    us = lambda x: x / 100.0  # 100 MHz ticks -> us
    t0 = s[:, 0].min()
    print("workgroups %d, kernel span %.1f us" % (a.n, us(s[:, 14].max() - t0)))
    print("per workgroup: total %.1f us (median)" % us(np.median(s[:, 14] - s[:, 0])))
    if s[:, 15].any():  # packed tabs: positions loaded and bucket-counted
        print("seg 0 sort: refs loaded + counted %.1f us, the rest of the sort %.1f us (medians)" %
              (us(np.median(s[:, 15] - s[:, 0])), us(np.median(s[:, 1] - s[:, 15]))))
    prev = s[:, 0]
    for seg in range(4):
        a1, a2, a3 = s[:, 1 + 3 * seg], s[:, 2 + 3 * seg], s[:, 3 + 3 * seg]
        print("seg %d: refs+lengths+scan %.1f  rows+lists %.1f  copy %.1f us (medians)" %
              (seg, us(np.median(a1 - prev)), us(np.median(a2 - a1)), us(np.median(a3 - a2))))
        prev = a3
    print("last partial chunks %.1f  headers/replay %.1f us" % (us(np.median(s[:, 13] - prev)),
                                                             us(np.median(s[:, 14] - s[:, 13]))))
    starts = np.sort(s[:, 0] - t0)
    print("workgroup start offsets (us): first 4 %s ... last 4 %s" % (us(starts[:4]), us(starts[-4:])))


if __name__ == "__main__":
    main()
