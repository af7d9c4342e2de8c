#!/usr/bin/env python3
"""Host-inclusive hashing: the staged pipeline (hipMemcpyAsync both ways,
SHF_HASH_MEM_HOST) against kernels that read keys from and write hashes to
page-locked host memory directly over PCIe (zero copy), plus the raw copy
rates (H2D alone, D2H alone, both at once on two streams).

    python tools/host_zero_copy_probe.py [--n 10000000]
"""
import argparse
import ctypes
import glob
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=10_000_000)
    p.add_argument("--reps", type=int, default=5)
    a = p.parse_args()
    import torch

    import sharedhashfile_amd as hb
    from sharedhashfile_amd.keygen import device_random_bytes

    dev = torch.device("cuda", 0)
    lib = hb.load()
    hip_so = sorted(glob.glob(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so*")))[0]
    hip = ctypes.CDLL(hip_so)
    n = a.n
    seed = hb.SEED if hasattr(hb, "SEED") else 12345

    keys = device_random_bytes(n * 16, 77, dev).cpu()
    pk = keys.pin_memory()
    po = torch.empty((n, 2), dtype=torch.int64).pin_memory()
    po2 = torch.empty((n, 2), dtype=torch.int64).pin_memory()

    def devptr(t):
        d = ctypes.c_void_p()
        rc = hip.hipHostGetDevicePointer(ctypes.byref(d), ctypes.c_void_p(t.data_ptr()), 0)
        if rc != 0:
            raise RuntimeError("hipHostGetDevicePointer failed: %d" % rc)
        return d.value

    dk, do = devptr(pk), devptr(po2)
    print("host ptr %x -> device ptr %x (same: %s)" % (pk.data_ptr(), dk, dk == pk.data_ptr()), flush=True)

    def timeit(fn, reps=a.reps):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts))

    st = torch.cuda.current_stream()
    res = {}
    t = timeit(lambda: hb._check(lib.shf_hash_batch_fixed(pk.data_ptr(), 16, n, seed, po.data_ptr(), hb.MEM_HOST), "staged"))
    res["staged_pinned"] = n / t
    t = timeit(lambda: hb._check(lib.shf_hash_batch_fixed_async(ctypes.c_void_p(dk), 16, n, seed, ctypes.c_void_p(do),
                                                                ctypes.c_void_p(st.cuda_stream)), "zero-copy"))
    res["zero_copy_pinned"] = n / t
    same = torch.equal(po, po2)
    print("zero-copy results equal staged: %s" % same, flush=True)

    # hybrid: keys H2D by copy engine in chunks, hashes written by the kernel straight to host memory
    streams = [torch.cuda.Stream() for _ in range(3)]
    for chunk in (1 << 20, 1 << 21, 1 << 22):
        dst = [torch.empty(chunk * 16, dtype=torch.uint8, device=dev) for _ in streams]
        po3 = torch.empty((n, 2), dtype=torch.int64).pin_memory()
        do3 = devptr(po3)
        flat = pk.view(-1)

        def hybrid():
            for ci, i0 in enumerate(range(0, n, chunk)):
                s = streams[ci % len(streams)]
                cnt = min(chunk, n - i0)
                with torch.cuda.stream(s):
                    dst[ci % len(streams)][:cnt * 16].copy_(flat[i0 * 16:(i0 + cnt) * 16], non_blocking=True)
                    hb._check(lib.shf_hash_batch_fixed_async(ctypes.c_void_p(dst[ci % len(streams)].data_ptr()), 16,
                                                             cnt, seed, ctypes.c_void_p(do3 + i0 * 16),
                                                             ctypes.c_void_p(s.cuda_stream)), "hybrid")
            for s in streams:
                s.synchronize()

        res["hybrid_h2d_copy_kernel_write_%dk" % (chunk >> 10)] = n / timeit(hybrid)
        same = same and torch.equal(po, po3)
    print("hybrid results equal staged: %s" % same, flush=True)

    # through the library (shf_hash_batch_fixed, MEM_HOST, page-locked buffers): staged vs zero copy
    for L in (16, 32, 48, 64, 128):
        m = max(1, (n * 16) // L)
        kb = device_random_bytes(m * L, 90 + L, dev).cpu().pin_memory()
        outs = {}
        for mode, env in (("staged", "0"), ("zero_copy", str(1 << 20))):
            os.environ["SHF_HB_ZERO_COPY_MAX_KEY"] = env
            o = torch.empty((m, 2), dtype=torch.int64).pin_memory()
            t = timeit(lambda: hb._check(lib.shf_hash_batch_fixed(kb.data_ptr(), L, m, seed, o.data_ptr(), hb.MEM_HOST),
                                         mode))
            res["lib_%s_%dB" % (mode, L)] = m / t
            outs[mode] = o
        same = same and torch.equal(outs["staged"], outs["zero_copy"])
    os.environ.pop("SHF_HB_ZERO_COPY_MAX_KEY")
    print("library zero-copy results equal staged: %s" % same, flush=True)

    # pageable caller buffers: staged pipeline vs registering them per call (hipHostRegister) + zero copy
    import numpy as _np
    pk_np = _np.ascontiguousarray(keys.numpy())
    out_np = _np.zeros((n, 2), dtype=_np.uint64)
    res["pageable_staged"] = n / timeit(lambda: hb._check(lib.shf_hash_batch_fixed(pk_np.ctypes.data, 16, n, seed,
                                                                                 out_np.ctypes.data, hb.MEM_HOST), "pg"))
    want = out_np.copy()

    def reg_call():
        for arr in (pk_np, out_np):
            rc = hip.hipHostRegister(ctypes.c_void_p(arr.ctypes.data), ctypes.c_size_t(arr.nbytes), 0)
            assert rc == 0, rc
        try:
            hb._check(lib.shf_hash_batch_fixed(pk_np.ctypes.data, 16, n, seed, out_np.ctypes.data, hb.MEM_HOST), "reg")
        finally:
            for arr in (pk_np, out_np):
                hip.hipHostUnregister(ctypes.c_void_p(arr.ctypes.data))

    out_np[:] = 0
    res["pageable_register_zero_copy"] = n / timeit(reg_call)
    same = same and _np.array_equal(out_np, want)
    print("register+zero-copy results equal staged: %s" % same, flush=True)

    dbuf = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    hbuf = torch.empty(n * 16, dtype=torch.uint8).pin_memory()
    nb = n * 16
    res["h2d_GBps"] = nb / timeit(lambda: dbuf.copy_(pk.view(-1), non_blocking=True)) / 1e9
    res["d2h_GBps"] = nb / timeit(lambda: hbuf.copy_(dbuf, non_blocking=True)) / 1e9
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    dbuf2 = torch.empty_like(dbuf)

    def both():
        with torch.cuda.stream(s1):
            dbuf2.copy_(pk.view(-1), non_blocking=True)
        with torch.cuda.stream(s2):
            hbuf.copy_(dbuf, non_blocking=True)
        s1.synchronize()
        s2.synchronize()

    res["h2d_plus_d2h_GBps_each"] = nb / timeit(both) / 1e9
    for k, v in res.items():
        print("%-24s %s" % (k, ("%.3f G keys/s" % (v / 1e9)) if "GBps" not in k else "%.1f GB/s" % v), flush=True)
    if not same:
        sys.exit(1)


if __name__ == "__main__":
    main()
