#!/usr/bin/env python3
"""Benchmark: device-resident batch key hashing on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

A "step" is one launch of the hashing kernel over one whole batch of synthetic
keys already resident in HBM (the batch is regenerated on device before timing,
never inside the timed region).

Headline (`value`): BASELINE.json configs[1] = 10M fixed 16-byte keys per GPU,
MurmurHash3_x64_128 seed 12345 (= shf_make_hash, /root/reference/src/shf.c:456)
-> 16-byte SHF_HASH per key. Also reported (`secondary`): configs[2] (100M x
256-byte keys) and configs[3] (100M variable-length keys, 8..512 B), and the
row pre-probe: the configs[1] keys hashed and probed against
a device row index holding all of them (`probe16`).

Multi-GPU: one process per GPU, each hashes its own independent shard (weak
scaling); torch.distributed (RCCL) is used only for the start/stop barriers and
the max-over-ranks of the elapsed time -- there is no collective on the data path.
"""
import argparse
import csv
import glob
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "keys hashed/s device-resident (16 B & 256 B keys) + GiB/s vs HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s HBM3E peak (spec)
SEED = 12345
WARMUP_MIN_S = 0.25  # untimed warmup floor per workload (seconds of GPU work)

# algorithmic bytes per key = key bytes read + 16-byte SHF_HASH
# written (+ 8-byte offset read for variable-length keys).
KERNEL_NAMES = {"fixed16": "k_fixed16", "tiled": "k_tiled", "generic": "k_generic"}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--keys16", type=int, default=10_000_000, help="configs[1]: 16-B keys per GPU")
    p.add_argument("--keys1b", type=int, default=1_000_000_000,
                   help="configs[4]: 16-B keys for the whole job, split over the GPUs (strong scaling)")
    p.add_argument("--keys256", type=int, default=100_000_000, help="configs[2]: 256-B keys per GPU")
    p.add_argument("--keysvar", type=int, default=100_000_000, help="configs[3]: 8..512-B keys per GPU")
    p.add_argument("--only", default="", help="comma list of fixed16,fixed256,var,probe16 (default: all)")
    p.add_argument("--probe-tabs", type=int, default=16, help="probe16: physical tabs per window in the index")
    p.add_argument("--var-kernel", default="auto", choices=["auto", "span", "generic", "round"])
    p.add_argument("--fixed-kernel", default="auto", choices=["auto", "fixed16", "tiled", "generic", "span"])
    p.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--cpu-threads", type=int, default=16, help="threads for cpu_baseline.all_cores (0/1: skip)")
    p.add_argument("--traffic", default="auto", choices=["auto", "off"],
                   help="auto: at N=1 run two short rocprofv3 --pmc child passes for HBM bytes")
    p.add_argument("--host-inclusive", action="store_true",
                   help="also time the pinned host->device->host path (reported, never `value`)")
    p.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                   help="backend for the barrier/max-reduce only (gloo: multi-rank rehearsal on one GPU)")
    p.add_argument("--warmup-min-s", type=float, default=WARMUP_MIN_S,
                   help="keep warming up (untimed) until this many seconds of the workload have run")
    p.add_argument("--quiet", action="store_true")
    return p.parse_args()


def dist_env():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return rank, world, local


def log(args, *a):
    if not args.quiet:
        print(*a, file=sys.stderr, flush=True)


# ---------------------------------------------------------------------------
# workloads
# ---------------------------------------------------------------------------
class Workload:
    """One device-resident batch and the launch that hashes it."""

    def __init__(self, name, n, bytes_per_key, launch, kernel, desc):
        self.name, self.n, self.bytes_per_key = name, n, bytes_per_key
        self.launch, self.kernel, self.desc = launch, kernel, desc


def fast_launch(hb, keys, key_len, n, out, kernel, dev):
    """The C-ABI launch with its ctypes arguments built once: a 50-us kernel must
    not wait on per-call Python argument checks (hb.hash_fixed does the same call)."""
    import ctypes

    import torch

    fn = hb.load().shf_hash_batch_fixed_kernel_async
    argv = (ctypes.c_void_p(keys.data_ptr()), ctypes.c_uint32(key_len), ctypes.c_uint64(n),
            ctypes.c_uint32(SEED), ctypes.c_void_p(out.data_ptr()), ctypes.c_int(kernel),
            ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream))

    def launch():
        rc = fn(*argv)
        if rc:
            raise hb.ShfHashBatchError(rc, "shf_hash_batch_fixed_kernel_async")

    return launch


def make_workloads(args, dev, rank, world=1):
    import torch

    import sharedhashfile_amd as hb
    from sharedhashfile_amd.keygen import device_random_bytes

    only = set(filter(None, args.only.split(","))) or {"fixed16", "fixed256", "var", "probe16", "shard1b"}
    wl = []
    seed_base = 0x5348460000000001 + 1000 * rank
    if "fixed16" in only:
        n = args.keys16
        keys = device_random_bytes(n * 16, seed_base + 1, dev)
        out = torch.empty((n, 2), dtype=torch.int64, device=dev)
        fk = {"auto": 0, "fixed16": 1, "tiled": 2, "generic": 3, "span": 4}[args.fixed_kernel]
        wl.append(Workload("fixed16", n, 16 + 16, fast_launch(hb, keys, 16, n, out, fk, dev),
                           "k_fixed16", "%d fixed 16-B keys" % n))
    if "shard1b" in only:
        # configs[4]: 1B 16-B keys split evenly over the job's GPUs (strong scaling:
        # 1B / world keys on this rank, contiguous index range, no collective).
        from sharedhashfile_amd.shard import shard_range

        total = args.keys1b
        lo, hi = shard_range(total, rank, world)
        n = hi - lo
        keys = device_random_bytes(n * 16, seed_base + 6, dev)
        out = torch.empty((n, 2), dtype=torch.int64, device=dev)
        w = Workload("shard1b", n, 16 + 16, fast_launch(hb, keys, 16, n, out, 0, dev),
                     "k_fixed16", "%d 16-B keys split over %d GPU(s): keys [%d, %d) on rank %d" % (total, world, lo, hi, rank))
        w.job_keys = total
        wl.append(w)
    if "fixed256" in only:
        n = args.keys256
        keys = device_random_bytes(n * 256, seed_base + 2, dev)
        out = torch.empty((n, 2), dtype=torch.int64, device=dev)
        fk = {"auto": 0, "fixed16": 2, "tiled": 2, "generic": 3, "span": 4}[args.fixed_kernel]
        wl.append(Workload("fixed256", n, 256 + 16,
                           lambda k=keys, o=out, fk=fk: hb.hash_fixed(k, 256, out=o, kernel=fk),
                           "k_tiled", "%d fixed 256-B keys" % n))
    if "var" in only:
        n = args.keysvar
        g = torch.Generator(device=dev)
        g.manual_seed(seed_base + 3)
        lens = torch.randint(8, 513, (n,), generator=g, device=dev, dtype=torch.int64)
        off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        torch.cumsum(lens, 0, out=off[1:])
        total = int(off[-1].item())
        data = device_random_bytes(total, seed_base + 4, dev)
        out = torch.empty((n, 2), dtype=torch.int64, device=dev)
        del lens
        wl.append(Workload("var", n, total / n + 8 + 16,
                           lambda d=data, o=off, out=out, vk={"auto": 0, "span": 4, "generic": 3, "round": 5}[args.var_kernel]:
                           hb.hash_var(d, o, out=out, kernel=vk, key_bytes=total),
                           {"generic": "k_generic", "round": "k_vround", "span": "k_span"}.get(args.var_kernel, "k_span"), "%d variable keys U[8,512] B, %.3f GB of key bytes" % (n, total / 1e9)))
    if "probe16" in only:
        # Row pre-probe: hash + row scan of every key against an index holding
        # all of them (a get-hit batch). Bytes per key: 16 key + 128 row +
        # 16 record; the 2 MiB tab map is read once per launch.
        from sharedhashfile_amd.rowindex import synthetic_index

        n = args.keys16
        keys = device_random_bytes(n * 16, seed_base + 5, dev)
        h = hb.hash_fixed(keys, 16)
        tab_slot, rows, n_slots, placed = synthetic_index(h, tabs_per_win=args.probe_tabs)
        index = hb.RowIndex(n_slots, tab_slot, rows)
        del h, tab_slot, rows
        out = torch.empty((n, 4), dtype=torch.int32, device=dev)
        wl.append(Workload("probe16", n, 16 + 128 + 16 + 4 * 256 * 2048 / n,
                           lambda k=keys, o=out, ix=index: hb.probe_fixed(ix, k, 16, out=o),
                           "k_fixed16<kOutProbe>", "%d fixed 16-B keys hashed and probed against a row index of "
                           "%d slots (%.0f MiB) holding %d of them" % (n, n_slots, n_slots / 16, placed)))
        wl[-1].index = index
    torch.cuda.synchronize()
    return wl


def time_workload(w, steps, warmup, dist, warmup_min_s=WARMUP_MIN_S):
    """Returns (wall seconds for `steps` steps, max over ranks; mean per-launch
    kernel seconds from HIP events on the launch stream)."""
    import torch

    stream = torch.cuda.current_stream()  # the stream every launch goes to (hb passes it to the library)
    # W warmup steps, continued (untimed) until the GPU has run this workload
    # for WARMUP_MIN_S: after seconds of host-side setup the clocks start low,
    # and 10 steps of a 50-us kernel are not enough to bring them up.
    t_w = time.perf_counter()
    done = 0
    while done < warmup or time.perf_counter() - t_w < warmup_min_s:
        w.launch()
        done += 1
        if done >= warmup and done % 16 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(steps):
        w.launch()
    ev1.record(stream)
    t_enq = time.perf_counter()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    w.enqueue_s = t_enq - t0  # host time to enqueue the steps (diagnostic)
    if dist:
        dist.barrier()
    elapsed = t1 - t0
    # HIP events bracketing the timed region on the launch stream: mean device
    # time per launch, back-to-back kernels (inter-kernel gaps included)
    per_launch = ev0.elapsed_time(ev1) / steps / 1e3
    if dist:
        dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
        t = torch.tensor([elapsed, per_launch], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, per_launch = float(t[0]), float(t[1])
    return elapsed, per_launch


def time_host_inclusive(args, n=10_000_000):
    """Host buffers in and out (SHF_HASH_MEM_HOST): H2D keys + kernel + D2H
    hashes, pipelined in SHF_HB_STAGE_MB chunks, SHF_HB_SLOTS in flight on their
    own streams. Pageable buffers are staged through pinned memory; page-locked
    ones are DMA'd directly."""
    import torch

    import sharedhashfile_amd as hb
    from sharedhashfile_amd.keygen import splitmix_bytes

    lib = hb.load()
    keys = np.frombuffer(splitmix_bytes(n * 16, 77), dtype=np.uint8).copy()
    res = {"keys": n, "key_len": 16, "unit": "keys/s"}
    pk = torch.from_numpy(keys).pin_memory()
    po = torch.empty((n, 2), dtype=torch.int64).pin_memory()
    out = np.empty((n, 2), dtype=np.uint64)
    for name, kp, op in [("pageable", keys.ctypes.data, out.ctypes.data), ("pinned", pk.data_ptr(), po.data_ptr())]:
        assert lib.shf_hash_batch_fixed(kp, 16, n, SEED, op, hb.MEM_HOST) == 0
        reps = 5
        t0 = time.perf_counter()
        for _ in range(reps):
            assert lib.shf_hash_batch_fixed(kp, 16, n, SEED, op, hb.MEM_HOST) == 0
        dt = (time.perf_counter() - t0) / reps
        res[name] = n / dt
    return res


# ---------------------------------------------------------------------------
# CPU baseline: the reference's own shf_make_hash() loop (test.9 shape)
# ---------------------------------------------------------------------------
def cpu_baseline(args):
    from sharedhashfile_amd.keygen import splitmix_bytes

    n, L = 1_000_000, 16  # BASELINE.json configs[0]: 1M 16-byte keys
    keys = np.frombuffer(splitmix_bytes(n * L, 0x5348460000000000), dtype=np.uint8).copy()
    try:
        from oracle.oracle_py import reference_lib

        ref = reference_lib()
    except Exception:
        ref = None
    import ctypes

    if ref is not None:
        fold = ctypes.c_uint64(0)
        dt1 = ref.ref_bench_make_hash_loop(keys.ctypes.data, L, n, 1, 1, ctypes.byref(fold))
        passes = max(1, int(args.cpu_seconds / max(dt1, 1e-6)))
        dt = ref.ref_bench_make_hash_loop(keys.ctypes.data, L, n, passes, 1, ctypes.byref(fold))
        kind = "reference"
        what = "oracle/_ref/libref_shf.so: reference src/shf.c shf_make_hash() + src/murmurhash3.c, gcc -O2"
    else:
        from oracle.oracle_py import Oracle

        o = Oracle()
        t0 = time.perf_counter()
        o.hash_fixed(keys, L)
        dt1 = time.perf_counter() - t0
        passes = max(1, int(args.cpu_seconds / max(dt1, 1e-6)))
        t0 = time.perf_counter()
        for _ in range(passes):
            o.hash_fixed(keys, L)
        dt = time.perf_counter() - t0
        kind = "port"
        what = "oracle/murmur3_oracle.c restatement, gcc -O2"
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            model = next((l.split(":", 1)[1].strip() for l in f if l.startswith("model name")), "")
    except OSError:
        pass
    out = {"value": n * passes / dt, "unit": "keys/s", "cores": 1, "kind": kind,
           "sample": "%d passes x 1M 16-B keys (test.9 loop shape, hash only), %.1f s, %s; host %s (%d cpus visible)"
                     % (passes, dt, what, model, os.cpu_count() or 0)}
    # SURVEY.md s8(d) config A also asks for all cores: the box's CPU share for one GPU is 16 threads
    threads = args.cpu_threads
    if threads > 1:
        mt_passes = max(1, int(passes * threads / 4))  # ~1/4 of the single-core time if it scales
        if ref is not None:
            dt_mt = ref.ref_bench_make_hash_loop(keys.ctypes.data, L, n, mt_passes, threads, ctypes.byref(fold))
        else:
            t0 = time.perf_counter()
            for _ in range(mt_passes):
                o.hash_fixed(keys, L, threads=threads)
            dt_mt = time.perf_counter() - t0
        out["all_cores"] = {"value": n * mt_passes / dt_mt, "unit": "keys/s", "cores": threads,
                            "sample": "%d passes x 1M 16-B keys over %d threads (even key ranges), %.1f s"
                                      % (mt_passes, threads, dt_mt)}
    return out


# ---------------------------------------------------------------------------
# HBM traffic from rocprofv3 PMC counters (child processes, N=1 only)
# ---------------------------------------------------------------------------
def collect_traffic(args, kernel_sym):
    """Two --pmc passes (FETCH_SIZE and WRITE_SIZE cannot share one pass on gfx950).
    Per MI355X_MICROARCH.md s HBM: FETCH_SIZE reads half the bytes of a wide
    coalesced stream on gfx950 -> doubled; both are in KiB."""
    prof = shutil.which("rocprofv3")
    if not prof:
        return None, "rocprofv3 not found"
    res = {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        outdir = tempfile.mkdtemp(prefix="shfhb_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
        cmd = [prof, "--pmc", counter, "--output-format", "csv", "-d", outdir, "-o", "pmc", "--",
               sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1", "--only", "fixed16",
               "--no-cpu", "--traffic", "off", "--quiet", "--keys16", str(args.keys16), "--warmup-min-s", "0"]
        try:
            subprocess.run(cmd, check=True, timeout=300, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                           cwd=os.environ.get("TMPDIR", "/tmp"))
        except Exception as e:  # noqa: BLE001
            return None, "rocprofv3 %s pass failed: %s" % (counter, e)
        vals = []
        for f in glob.glob(os.path.join(outdir, "**", "*counter_collection*.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    if kernel_sym in row.get("Kernel_Name", "") and row.get("Counter_Name") == counter:
                        vals.append(float(row["Counter_Value"]))
        shutil.rmtree(outdir, ignore_errors=True)
        if not vals:
            return None, "no %s rows for %s" % (counter, kernel_sym)
        res[counter] = float(np.median(vals))
    fetch = 2.0 * res["FETCH_SIZE"] * 1024.0
    write = res["WRITE_SIZE"] * 1024.0
    return fetch + write, "per launch: 2 x FETCH_SIZE (%.0f KiB) + WRITE_SIZE (%.0f KiB), median of 3 launches" % (
        res["FETCH_SIZE"], res["WRITE_SIZE"])


def main():
    args = parse()
    rank, world, local = dist_env()
    import torch

    import sharedhashfile_amd as hb

    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU (HIP); none visible")
    local = local % max(1, torch.cuda.device_count())  # ranks beyond the visible GPUs share them (rehearsal)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as tdist

        if args.dist_backend == "nccl":  # RCCL: barriers + one max-reduce, no data path
            tdist.init_process_group("nccl", device_id=dev)
        else:
            tdist.init_process_group("gloo")
        dist = tdist
    hb.check_device()

    wl = make_workloads(args, dev, rank, world)
    results = {}
    for w in wl:
        elapsed, per_launch = time_workload(w, args.steps, args.warmup, dist, args.warmup_min_s)
        keys_total = getattr(w, "job_keys", w.n * world) * args.steps
        results[w.name] = {
            "value": keys_total / elapsed,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "kernel_us": per_launch * 1e6,
            "achieved_gbs": w.n * w.bytes_per_key / per_launch / 1e9,
            "bytes_per_key": w.bytes_per_key,
            "kernel": w.kernel,
            "desc": w.desc,
            "enqueue_us_per_step": 1e6 * w.enqueue_s / args.steps,
        }
        log(args, "[bench] %s: %.3f Gkeys/s, %.1f us/launch, %.0f GB/s, host enqueue %.1f us/step" % (
            w.name, results[w.name]["value"] / 1e9, per_launch * 1e6, results[w.name]["achieved_gbs"],
            1e6 * w.enqueue_s / args.steps))

    if rank == 0:
        head = results.get("fixed16") or next(iter(results.values()))
        traffic, traffic_note = None, "not collected"
        if world == 1 and args.traffic == "auto" and "fixed16" in results:
            traffic, traffic_note = collect_traffic(args, "k_fixed16")
        roof = {"bound": "hbm", "achieved": round(head["achieved_gbs"], 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(head["achieved_gbs"] / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "kernel": head["kernel"], "kernel_us": round(head["kernel_us"], 2),
                "algorithmic_bytes_per_launch": int(args.keys16 * 32) if "fixed16" in results else None,
                "traffic_note": traffic_note}
        cpu = None
        if world == 1 and not args.no_cpu:
            cpu = cpu_baseline(args)
        secondary = {}
        for name, r in results.items():
            if name == "fixed16":
                continue
            secondary[name] = {"value": r["value"], "unit": "keys/s", "ms_per_step": round(r["ms_per_step"], 4),
                               "desc": r["desc"], "kernel": r["kernel"], "kernel_us": round(r["kernel_us"], 2),
                               "roofline": {"bound": "hbm", "achieved": round(r["achieved_gbs"], 1),
                                            "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                            "frac": round(r["achieved_gbs"] / HBM_PEAK_GBS, 4),
                                            "bytes_per_key": round(r["bytes_per_key"], 2)}}
            if name == "shard1b":
                secondary[name]["scaling"] = "strong"
        line = {
            "metric": METRIC,
            "value": head["value"],
            "unit": "keys/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": head["ms_per_step"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic: random key bytes generated on device (torch Philox), resident in HBM before timing",
            "config": {"workload": "BASELINE configs[1]: %d fixed 16-B keys per GPU, MurmurHash3_x64_128 seed "
                                   "12345 -> 16-B SHF_HASH (shf_make_hash batch)" % args.keys16,
                       "keys_per_gpu": args.keys16, "key_len": 16,
                       "parallelism": "dp%d (independent key shards, no collective)" % world},
            "roofline": roof,
            "cpu_baseline": cpu,
            "secondary": secondary,
        }
        if args.host_inclusive and world == 1:
            line["host_inclusive"] = time_host_inclusive(args)
        print(json.dumps(line), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
