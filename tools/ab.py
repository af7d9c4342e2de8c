#!/usr/bin/env python3
"""Interleaved A/B timing of library build variants in ONE process
(cdna_hip_programming.md s5.4 rule 24).

    python tools/ab.py --variant base= --variant exp=@tools/_ab/lib_exp.so \
        --workload var --n 25000000 --rounds 8

`name=` is the in-tree build; `name=@path.so` a library built beforehand on
the CPU host from an experimental copy of the sources (the library itself has
no compile-time alternatives: tests/test_abi.py); `name=-Dflags` builds the
in-tree sources with extra flags. The variants are loaded side by side through
ctypes; every round times every variant once.
"""
import argparse
import ctypes
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def build(name, flags, outdir):
    from sharedhashfile_amd import build as b

    if flags.startswith("@"):  # prebuilt variant (tools/ab.py --prebuild on the CPU host)
        return os.path.join(ROOT, flags[1:])

    if not flags.strip() and os.path.exists(os.path.join(ROOT, "sharedhashfile_amd", "libshf_hash_batch.so")):
        return os.path.join(ROOT, "sharedhashfile_amd", "libshf_hash_batch.so")  # the in-tree build as is

    so = os.path.join(outdir, "lib_%s.so" % name)
    cmd = [b.hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-fvisibility=hidden",
           "-I" + os.path.join(ROOT, "include")] + flags.split() + [os.path.join(b.CSRC, s) for s in b.SOURCES] + [
               "-o", so]
    subprocess.check_call(cmd)
    return so


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--variant", action="append", required=True, help="name=-Dflags ...")
    p.add_argument("--workload", default="fixed256", choices=["fixed16", "fixed256", "var", "fixedL", "probe16", "probeh", "tab"])
    p.add_argument("--key-len", type=int, default=37)
    p.add_argument("--n", type=int, default=20_000_000)
    p.add_argument("--rounds", type=int, default=6)
    p.add_argument("--reps", type=int, default=5)
    p.add_argument("--kernel", type=int, default=0)
    p.add_argument("--var-lo", type=int, default=8, help="var workload: key lengths U[var-lo, var-hi]")
    p.add_argument("--var-hi", type=int, default=512)
    p.add_argument("--copy-ref", action="store_true", help="also time torch copy_ of the same byte count")
    p.add_argument("--sized", action="store_true", help="var: pass the batch byte count (sized-window API)")
    p.add_argument("--sort-chunk", type=int, default=0,
                   help="var: sort the key lengths within chunks of this many keys (what length bucketing buys)")
    p.add_argument("--warmup-s", type=float, default=1.0, help="untimed calls of every variant for this long first")
    p.add_argument("--unchecked", action="append", default=[], help="variant whose results are not compared (ceilings)")
    p.add_argument("--prebuild", default="", help="build every name=-Dflags variant into this dir and exit")
    a = p.parse_args()
    if a.prebuild:
        os.makedirs(a.prebuild, exist_ok=True)
        for v in a.variant:
            name, _, flags = v.partition("=")
            print(build(name, flags, a.prebuild))
        return

    import torch

    import sharedhashfile_amd as hb
    from sharedhashfile_amd.keygen import device_random_bytes

    def cs():  # the current stream's handle
        return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    outdir = tempfile.mkdtemp(prefix="shfhb_ab_")
    libs = {}
    for v in a.variant:
        name, _, flags = v.partition("=")
        libs[name] = hb.load(build(name, flags, outdir))
    dev = torch.device("cuda:0")
    n = a.n
    out_shape = (n, 2)
    if a.workload in ("probe16", "probeh"):  # hash+probe / probe of hashes against an index of all keys
        from sharedhashfile_amd.rowindex import synthetic_index

        keys = device_random_bytes(n * 16, 1, dev)
        h = hb.hash_fixed(keys, 16)
        ts, rows, n_slots, _ = synthetic_index(h, tabs_per_win=16)
        index = hb.RowIndex(n_slots, ts, rows)  # one handle; every variant reads the same device index
        del ts, rows
        out_shape = (n, 4)
        if a.workload == "probe16":
            per_key = 16 + 128 + 16
            call = lambda lib, out: lib.shf_probe_batch_fixed_kernel_async(index.handle, keys.data_ptr(), 16, n, 12345,
                                                                           None, out.data_ptr(), a.kernel, cs())
        else:
            per_key = 16 + 128 + 16
            call = lambda lib, out: lib.shf_probe_batch_hashes_async(index.handle, h.data_ptr(), n, out.data_ptr(),
                                                                     None)
    elif a.workload == "tab":  # f4: the bench's tab-part batch (bench.py tab_workload), a.n tabs
        import bench

        class _A:
            tab_jobs = a.n

        tw = bench.tab_workload(_A, dev, 0x5348460000000001)
        src, dst, d_jobs, d_maps, prm = tw.keep
        per_key = tw.bytes_per_key
        out_shape = None

        def call(lib, out):
            return lib.shf_tab_copy_batch_async(ctypes.c_void_p(src.data_ptr()), src.numel(),
                                                ctypes.c_void_p(out.data_ptr()), out.numel(),
                                                ctypes.c_void_p(d_jobs.data_ptr()), n, ctypes.c_void_p(d_maps.data_ptr()),
                                                8, ctypes.byref(prm), cs())
    elif a.workload in ("fixed16", "fixed256", "fixedL"):
        L = {"fixed16": 16, "fixed256": 256, "fixedL": a.key_len}[a.workload]
        keys = device_random_bytes(n * L, 1, dev)
        per_key = L + 16
        call = lambda lib, out: lib.shf_hash_batch_fixed_kernel_async(keys.data_ptr(), L, n, 12345, out.data_ptr(),
                                                                       a.kernel, cs())
    else:
        g = torch.Generator(device=dev)
        g.manual_seed(3)
        lens = torch.randint(a.var_lo, a.var_hi + 1, (n,), generator=g, device=dev, dtype=torch.int64)
        if a.sort_chunk:
            c = a.sort_chunk
            m = n // c * c
            lens[:m] = torch.sort(lens[:m].view(-1, c), dim=1).values.reshape(-1)
        off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        torch.cumsum(lens, 0, out=off[1:])
        data = device_random_bytes(int(off[-1].item()), 2, dev)
        per_key = float(off[-1].item()) / n + 24
        total = int(off[-1].item())
        if a.sized:
            call = lambda lib, out: lib.shf_hash_batch_var_sized_kernel_async(data.data_ptr(), off.data_ptr(), n, total,
                                                                               12345, out.data_ptr(), a.kernel, cs())
        else:
            call = lambda lib, out: lib.shf_hash_batch_var_kernel_async(data.data_ptr(), off.data_ptr(), n, 12345,
                                                                         out.data_ptr(), a.kernel, cs())
    if out_shape is None:  # tab: each variant writes its own copy of the output images
        outs = {k: torch.zeros_like(dst) for k in libs}
    else:
        outs = {k: torch.empty(out_shape, dtype=torch.int64 if out_shape[1] == 2 else torch.int32, device=dev)
                for k in libs}
    for k, lib in libs.items():
        assert call(lib, outs[k]) == 0
    torch.cuda.synchronize()
    ref = next(iter(outs.values()))
    for k, o in outs.items():
        assert k in a.unchecked or torch.equal(o, ref), "variant %s differs" % k
    if a.copy_ref:  # a known-good streaming reference on the same device: bytes in == bytes out
        half = int(n * per_key) // 2
        src_c = torch.empty(half, dtype=torch.uint8, device=dev)
        dst_c = torch.empty_like(src_c)
        libs["copy_ref"] = None
        outs["copy_ref"] = None
        call_orig = call
        call = lambda lib, out: (dst_c.copy_(src_c), 0)[1] if lib is None else call_orig(lib, out)
    t_end = time.time() + a.warmup_s  # clocks and caches settle before the timed rounds
    while time.time() < t_end:
        for k, lib in libs.items():
            call(lib, outs[k])
        torch.cuda.synchronize()
    times = {k: [] for k in libs}
    for r in range(a.rounds):
        for k, lib in libs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(a.reps):
                call(lib, outs[k])
            e1.record()
            e1.synchronize()
            times[k].append(e0.elapsed_time(e1) / a.reps)
    for k, ts in times.items():
        ts = sorted(ts)
        med = ts[len(ts) // 2]
        what = "M tabs/s" if a.workload == "tab" else "G keys/s"
        rate = n / med / (1e3 if a.workload == "tab" else 1e6)
        print("%-12s median %8.3f ms  min %8.3f ms  %7.1f GB/s  %6.2f %s" % (
            k, med, ts[0], n * per_key / med / 1e6, rate, what))


if __name__ == "__main__":
    main()
