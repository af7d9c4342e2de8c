#!/usr/bin/env python3
"""Benchmark: device-resident batch key hashing on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

A "step" is one launch of the hashing kernel over one whole batch of synthetic
keys already resident in HBM (batches are generated on device before the timed
region, never inside it).

Headline (`value`): BASELINE.json configs[1] = 10M fixed 16-byte keys per GPU,
MurmurHash3_x64_128 seed 12345 (= shf_make_hash, /root/reference/src/shf.c:456)
-> 16-byte SHF_HASH per key. The timed steps rotate over --rotate distinct
batches (keys + outputs, 4 x 320 MB by default), so no step re-reads lines the
previous step left in the 256 MiB Infinity Cache; the single-batch figure is
the secondary `fixed16_hot`. Also reported (`secondary`): configs[4]'s 1B keys
split over the job's GPUs (`shard1b`, strong scaling), configs[2] (100M x
256-byte keys), configs[3] (100M variable-length keys, 8..512 B), and the row
pre-probe (`probe16`).

Every line: min / median / max over --repeats timed repeats of K steps each
(`value` is the median), and after the timed region >= 20 000 sampled outputs
of the timed batches are checked against the CPU oracle (the checker only;
`verified`).

Ceilings measured in the same run on the same box (`secondary.ceil_*`,
include/shf_hash_batch_ceiling.h): a 16-B/lane copy in k_fixed16's launch shape
on the headline's own rotating buffers (and on the hot batch and the 1B-key
buffers), a 16:1 read-mostly copy on configs[2]'s buffers, the probe's 128-B
row gather and an unaligned 16-B stream. Every `roofline.frac_of_copy_ceiling`
divides by the ceiling of the matching shape measured here, never by a
constant; the gathers and the unaligned stream also calibrate rocprofv3's
FETCH_SIZE for the probe and the tab copy, and two VALU-saturating launches
calibrate the VALUBusy formula (`valu_busy`).

Multi-GPU: one process per GPU, each hashes its own
independent shard (no collective on the data path; torch.distributed is used
only for the start/stop barriers and the max over ranks of the elapsed time).
`--gpus N` without a torch.distributed launcher spawns the N rank processes
itself before anything touches the GPU. Each rank needs a GPU of its own; a
run with more ranks than visible GPUs is refused unless --allow-shared-gpu is
given, and then the line says `"rehearsal": true` and `n_gpus` counts the
distinct GPUs actually used.
"""
import argparse
import csv
import ctypes
import glob
import json
import os
import shutil
import socket
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "keys hashed/s device-resident (16 B & 256 B keys) + GiB/s vs HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s HBM3E peak (spec)
SIMDS = 256 * 4        # 256 CUs x 4 SIMDs
XCDS = 8
SEED = 12345
WARMUP_MIN_S = 0.25  # untimed warmup floor per workload (seconds of GPU work)
VERIFY_SAMPLES = 20_000
BOX_CPU_SHARE = 16   # host threads per GPU on the GPU box (its sizing rule for worker pools)

# rocprofv3 kernel-name substrings of each workload's kernel (PMC passes; rows
# are also matched on the launch's grid size, Workload.grid)
KERNEL_SYMS = {"fixed16": "k_fixed16<0>", "fixed16_hot": "k_fixed16<0>", "shard1b": "k_fixed16<0>",
               "fixed256": "k_tiled<0, 8>", "var": "k_span_pp<0", "probe16": "k_fixed16<2>", "probe16_hbm": "k_fixed16<2>",
               "tabpart": "k_tab_split", "ceil_copy": "k_ceil_copy(", "ceil_copy_hot": "k_ceil_copy(",
               "ceil_copy_1b": "k_ceil_copy(", "ceil_read16": "k_ceil_read16<false", "ceil_read16nt": "k_ceil_read16<true, 256",
               "ceil_read16w1": "k_ceil_read16<true, 64", "ceil_gather128": "k_ceil_gather128<false>",
               "ceil_stream16u": "k_ceil_stream16u", "ceil_valu_add": "k_ceil_valu<0>",
               "ceil_valu_mul": "k_ceil_valu<1>", "ceil_copynt": "k_ceil_copyv<1>(", "ceil_copynt_hot": "k_ceil_copyv<1>(",
               "ceil_copynt_1b": "k_ceil_copyv<1>(", "ceil_probe_rows": "k_ceil_gather128<true>",
               "ceil_probe_rows_hbm": "k_ceil_gather128<true>",
               "winorder": "k_wo_", "hashwin16": "k_fixed16_win"}
# workloads whose one call is several kernels: their counters are summed over the kernels
# (each kernel's median per launch), so traffic covers the whole call
MULTI_KERNEL = {"winorder": ["k_wo_rank", "k_wo_scan_rows", "k_wo_place"],
                "hashwin16": ["k_fixed16_win", "k_wo_scan_rows", "k_wo_place"]}
HASH_WORKLOADS = ["fixed16", "fixed16_hot", "shard1b", "fixed256", "var", "probe16", "probe16_hbm", "tabpart",
                  "winorder", "hashwin16"]
CEIL_WORKLOADS = ["ceil_copy", "ceil_copynt", "ceil_copy_hot", "ceil_copynt_hot", "ceil_copy_1b", "ceil_copynt_1b",
                  "ceil_read16", "ceil_read16nt", "ceil_read16w1", "ceil_probe_rows", "ceil_probe_rows_hbm", "ceil_gather128", "ceil_stream16u", "ceil_valu_add",
                  "ceil_valu_mul"]
# the ceiling each hashing line is reported against: the best copy of the same bytes on the same buffers
# (one lane per 16 B as k_fixed16 moves them, plain or nontemporal stores), measured in this run right after
# the line
CEILING_OF = {"fixed16": ["ceil_copy", "ceil_copynt"], "fixed16_hot": ["ceil_copy_hot", "ceil_copynt_hot"],
              "shard1b": ["ceil_copy_1b", "ceil_copynt_1b"], "fixed256": ["ceil_read16", "ceil_read16nt", "ceil_read16w1"],
              "var": ["ceil_read16", "ceil_read16nt", "ceil_read16w1"],
              "probe16": ["ceil_probe_rows"], "probe16_hbm": ["ceil_probe_rows_hbm"], "tabpart": ["ceil_copy", "ceil_copynt"],
              "winorder": ["ceil_copy", "ceil_copynt"], "hashwin16": ["ceil_copy", "ceil_copynt"]}
# timing order: each ceiling right after the line it bounds (same buffers, same thermal state)
ORDER = ["fixed16", "ceil_copy", "ceil_copynt", "fixed16_hot", "ceil_copy_hot", "ceil_copynt_hot", "shard1b",
         "ceil_copy_1b", "ceil_copynt_1b", "fixed256", "ceil_read16", "ceil_read16nt", "ceil_read16w1", "var", "probe16", "ceil_probe_rows",
         "probe16_hbm", "ceil_probe_rows_hbm",
         "ceil_gather128", "tabpart", "ceil_stream16u", "winorder", "hashwin16", "ceil_valu_add",
         "ceil_valu_mul"]
# the pattern whose known byte count calibrates each line's FETCH_SIZE
FETCH_CAL_OF = {"fixed16": "ceil_copy", "fixed16_hot": "ceil_copy", "shard1b": "ceil_copy",
                "fixed256": "ceil_read16", "var": "ceil_read16", "probe16": "ceil_gather128",
                "probe16_hbm": "ceil_gather128",
                "tabpart": "ceil_stream16u", "winorder": "ceil_copy", "hashwin16": "ceil_copy"}
# bytes per lane the ceiling kernels read and write (include/shf_hash_batch_ceiling.h)
CEIL_READ_PER_LANE = {"ceil_copy": 16, "ceil_copynt": 16, "ceil_read16": 256, "ceil_read16nt": 256, "ceil_read16w1": 256,
                      "ceil_gather128": 132,
                      "ceil_stream16u": 16}
VALU_ITERS = 2048          # rounds of 8 chained VALU ops per lane in the VALU-saturating launches
VALU_LANES = 256 * 32 * 64  # 32 waves per CU on 256 CUs


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None, help="GPUs (= ranks); default WORLD_SIZE or 1")
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--repeats", type=int, default=3, help="timed repeats of --steps steps per line")
    p.add_argument("--rotate", type=int, default=4, help="distinct 10M-key batches the headline rotates over")
    p.add_argument("--keys16", type=int, default=10_000_000, help="configs[1]: 16-B keys per GPU")
    p.add_argument("--keys1b", type=int, default=1_000_000_000,
                   help="configs[4]: 16-B keys for the whole job, split over the GPUs (strong scaling)")
    p.add_argument("--keys256", type=int, default=100_000_000, help="configs[2]: 256-B keys per GPU")
    p.add_argument("--keysvar", type=int, default=100_000_000, help="configs[3]: 8..512-B keys per GPU")
    p.add_argument("--only", default="", help="comma list of %s, %s" % (",".join(HASH_WORKLOADS),
                                                                           ",".join(CEIL_WORKLOADS)))
    p.add_argument("--probe-tabs", type=int, default=16,
                   help="probe16: physical tabs per window in the index (16: 256 MiB of rows, cache-resident)")
    p.add_argument("--probe-tabs-hbm", type=int, default=128,
                   help="probe16_hbm: tabs per window (128: 2 GiB of rows, well past the 256 MiB Infinity Cache)")
    p.add_argument("--tab-jobs", type=int, default=1024, help="tabpart: tabs parted per step (f4)")
    p.add_argument("--var-kernel", default="auto", choices=["auto", "span", "span_pp", "generic", "round"])
    p.add_argument("--fixed-kernel", default="auto", choices=["auto", "fixed16", "tiled", "generic", "span"])
    p.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-verify", action="store_true", help="skip the sampled oracle check of the timed outputs")
    p.add_argument("--traffic", default="auto", choices=["auto", "off"],
                   help="auto: at N=1 run rocprofv3 --pmc child passes (HBM bytes, VALU busy) per kernel")
    p.add_argument("--no-host-inclusive", action="store_true",
                   help="skip the host-buffer (pinned/pageable hipMemcpyAsync both ways) leg at N=1")
    p.add_argument("--host-keys", type=int, default=10_000_000, help="keys per host-inclusive batch")
    p.add_argument("--allow-shared-gpu", action="store_true",
                   help="rehearsal only: let ranks share GPUs (gloo barriers; the line is marked rehearsal)")
    p.add_argument("--dist-backend", default="gloo", choices=["gloo", "nccl"],
                   help="backend of the start/stop barriers and the max-over-ranks reduce only (no data crosses "
                        "GPUs): gloo on CPU tensors by default, RCCL on request")
    p.add_argument("--warmup-min-s", type=float, default=WARMUP_MIN_S,
                   help="keep warming up (untimed) until this many seconds of the workload have run")
    p.add_argument("--quiet", action="store_true")
    p.add_argument("--detail-out", default=None,
                   help="file for the full record (PMC, calibration, per-rank); default gpurun_out/bench_detail_nN.json")
    return p.parse_args(argv)


def log(args, *a):
    if not args.quiet:
        print(*a, file=sys.stderr, flush=True)


# ---------------------------------------------------------------------------
# launch: one process per GPU
# ---------------------------------------------------------------------------
def dist_env():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    return rank, world, local, local_world


def plan_device(local_rank, local_world, device_count, allow_shared):
    """(device index, shared) for this rank: one distinct GPU per local rank, or
    a refusal. Sharing (rank i on GPU i % count) only with allow_shared."""
    if device_count < 1:
        raise SystemExit("bench.py needs a GPU (HIP); none visible")
    if local_world > device_count:
        if not allow_shared:
            raise SystemExit("bench.py: %d ranks on this node but only %d GPU(s) visible; every rank needs a GPU "
                             "of its own (pass --allow-shared-gpu for a rehearsal, marked as such)"
                             % (local_world, device_count))
        return local_rank % device_count, True
    return local_rank, False


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def rank_envs(n, port, base=None):
    """The environment of each of n rank processes on this node (one GPU each)."""
    base = dict(os.environ if base is None else base)
    return [dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port)) for r in range(n)]


def launch_ranks(argv, n):
    """Start n rank processes of this script (RANK/WORLD_SIZE/... in their
    environment) and wait for them. This process never touches the GPU: the
    ranks are children, not an exec of a GPU-initialised process. The first
    rank to fail stops the others (by PID)."""
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env)
             for env in rank_envs(n, _free_port())]
    rc = 0
    while procs:
        for p in list(procs):
            code = p.poll()
            if code is None:
                continue
            procs.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in procs:
                    q.terminate()
        time.sleep(0.05)
    return rc


# ---------------------------------------------------------------------------
# workloads
# ---------------------------------------------------------------------------
class Workload:
    """Device-resident batches and the launch that hashes one of them.
    launch(i) hashes batch i % len(batches) into its own output."""

    def __init__(self, name, n, bytes_per_key, launches, kernel, desc, verify=None, grid=None):
        self.name, self.n, self.bytes_per_key = name, n, bytes_per_key
        self.launches, self.kernel, self.desc, self.verify = launches, kernel, desc, verify
        self.grid = grid  # work-items of one launch of the measured kernel (matches rocprofv3's Grid_Size)
        self.job_keys = None

    def launch(self, i):
        self.launches[i % len(self.launches)]()


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


def _sample_idx(n, k, seed):
    rng = np.random.default_rng(seed)
    idx = rng.integers(0, n, size=min(k, n), dtype=np.int64)
    return np.unique(np.concatenate([idx, [0, n - 1]]))


def verify_fixed(pairs, key_len, samples, seed):
    """pairs: [(keys, out)] device tensors. Sampled keys of every pair, hashed
    by the CPU oracle (the checker), against the timed outputs."""
    import torch

    from oracle.oracle_py import Oracle

    o = Oracle()
    per = max(1, samples // len(pairs))
    checked = 0
    for j, (keys, out) in enumerate(pairs):
        n = out.shape[0]
        idx = _sample_idx(n, per, seed + j)
        ti = torch.from_numpy(idx).to(keys.device)
        k = keys.view(n, key_len).index_select(0, ti).cpu().numpy()
        got = out.index_select(0, ti).cpu().numpy().view(np.uint64)
        if not np.array_equal(got, o.hash_fixed(k, key_len)):
            return False, checked
        checked += idx.size
    return True, checked


def verify_var(data, off, out, samples, seed):
    import torch

    from oracle.oracle_py import Oracle

    n = out.shape[0]
    idx = _sample_idx(n, samples, seed)
    ti = torch.from_numpy(idx).to(data.device)
    o0, o1 = off.index_select(0, ti), off.index_select(0, ti + 1)
    lens = o1 - o0
    starts = torch.repeat_interleave(o0, lens)
    first = torch.repeat_interleave(torch.cumsum(lens, 0) - lens, lens)
    pos = starts + (torch.arange(starts.numel(), device=data.device) - first)
    sub = data[pos].cpu().numpy()
    hoff = np.zeros(idx.size + 1, dtype=np.uint64)
    hoff[1:] = np.cumsum(lens.cpu().numpy())
    got = out.index_select(0, ti).cpu().numpy().view(np.uint64)
    return bool(np.array_equal(got, Oracle().hash_var(sub, hoff))), int(idx.size)


def _up(x, m):
    return (x + m - 1) // m * m


def grid_threads(name, n):
    """Work-items of one launch of workload `name` over n keys / lanes / jobs:
    rocprofv3's Grid_Size of that launch (the PMC rows are matched on it)."""
    if name == "ceil_read16w1":
        return n                        # one 64-thread workgroup per 64 lanes (n a multiple of 64)
    if name in ("fixed16", "fixed16_hot", "shard1b", "probe16", "probe16_hbm") or name.startswith("ceil_"):
        return _up(n, 256)              # 256-thread blocks, one key / lane per thread
    if name == "fixed256":
        return _up(n, 64)               # k_tiled: one 64-thread workgroup per 64-key tile
    if name == "var":
        return ((n + 63) // 64 + 1) // 2 * 128  # k_span_pp: one 128-thread workgroup per two tiles
    if name == "tabpart":
        return n * 512                  # k_tab_split: one 512-thread workgroup per tab
    if name in ("winorder", "hashwin16"):
        return (n + 4095) // 4096 * 256  # k_wo_rank: one 256-thread workgroup per 4096 keys
    return None


def read16_lanes(args, only):
    """Lanes of the read-mostly ceiling: configs[2]'s keys when that line runs (its own buffers), else 10M."""
    n = args.keys256 if "fixed256" in only else min(args.keys256, 10_000_000)
    return n - n % 64


def ceil_launcher(hb, kind, src, src_bytes, idx, dst, n, dev):
    """shf_hb_ceiling_async (include/shf_hash_batch_ceiling.h) with its ctypes arguments built once."""
    import ctypes

    import torch

    from sharedhashfile_amd import bench_ceiling

    fn = bench_ceiling.load().shf_hb_ceiling_async
    argv = (ctypes.c_int(kind), ctypes.c_void_p(src), ctypes.c_uint64(src_bytes), ctypes.c_void_p(idx or 0),
            ctypes.c_void_p(dst), ctypes.c_uint64(n), ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream))

    def launch():
        rc = fn(*argv)
        if rc:
            raise hb.ShfHashBatchError(rc, "shf_hb_ceiling_async(%d)" % kind)

    return launch


def make_workloads(args, dev, rank, world=1):
    import torch

    import sharedhashfile_amd as hb
    from sharedhashfile_amd.keygen import device_random_bytes

    only = set(filter(None, args.only.split(","))) or set(HASH_WORKLOADS + CEIL_WORKLOADS)
    wl = []
    seed_base = 0x5348460000000001 + 1000 * rank
    fk16 = {"auto": 0, "fixed16": 1, "tiled": 2, "generic": 3, "span": 4}[args.fixed_kernel]
    bufs = {}

    def fixed16_pairs():  # configs[1]'s rotating batches (keys + outputs), shared by its copy ceiling
        if "pairs" not in bufs:
            n = args.keys16
            bufs["pairs"] = [(device_random_bytes(n * 16, seed_base + 1 + 100 * b, dev),
                              torch.empty((n, 2), dtype=torch.int64, device=dev)) for b in range(max(1, args.rotate))]
        return bufs["pairs"]

    if "fixed16" in only or "fixed16_hot" in only:
        n = args.keys16
        pairs = fixed16_pairs()
        B = len(pairs)
        if "fixed16" in only:
            wl.append(Workload("fixed16", n, 16 + 16, [fast_launch(hb, k, 16, n, o, fk16, dev) for k, o in pairs],
                               "k_fixed16", "%d fixed 16-B keys per step, rotating over %d distinct batches "
                               "(%.2f GB of keys + hashes)" % (n, B, B * n * 32 / 1e9),
                               lambda p=pairs: verify_fixed(p, 16, VERIFY_SAMPLES, 11), grid_threads("fixed16", n)))
        if "fixed16_hot" in only:
            k0, o0 = pairs[0]
            wl.append(Workload("fixed16_hot", n, 16 + 16, [fast_launch(hb, k0, 16, n, o0, fk16, dev)], "k_fixed16",
                               "%d fixed 16-B keys, the same batch every step (its 320 MB partly stay in the "
                               "256 MiB Infinity Cache)" % n,
                               lambda p=pairs[:1]: verify_fixed(p, 16, VERIFY_SAMPLES, 12),
                               grid_threads("fixed16_hot", n)))
    if "shard1b" in only or "ceil_copy_1b" in only or "ceil_copynt_1b" in only:
        # configs[4]: 1B 16-B keys split evenly over the job's GPUs (strong scaling:
        # 1B / world keys on this rank, contiguous index range, no collective).
        from sharedhashfile_amd.shard import shard_range

        total = args.keys1b
        lo, hi = shard_range(total, rank, world)
        n = hi - lo
        keys = device_random_bytes(n * 16, seed_base + 6, dev)
        out = torch.empty((n, 2), dtype=torch.int64, device=dev)
        bufs["shard1b"] = (keys, out, n)
        if "shard1b" in only:
            w = Workload("shard1b", n, 16 + 16, [fast_launch(hb, keys, 16, n, out, 0, dev)], "k_fixed16",
                         "%d 16-B keys split over %d rank(s): keys [%d, %d) on rank %d" % (total, world, lo, hi, rank),
                         lambda p=[(keys, out)]: verify_fixed(p, 16, VERIFY_SAMPLES, 13), grid_threads("shard1b", n))
            w.job_keys = total
            w.shard = (lo, hi)
            wl.append(w)
    if "fixed256" in only:
        n = args.keys256
        keys = device_random_bytes(n * 256, seed_base + 2, dev)
        out = torch.empty((n, 2), dtype=torch.int64, device=dev)
        bufs["fixed256"] = (keys, out, n)
        fk = {"auto": 0, "fixed16": 2, "tiled": 2, "generic": 3, "span": 4}[args.fixed_kernel]
        wl.append(Workload("fixed256", n, 256 + 16, [fast_launch(hb, keys, 256, n, out, fk, dev)],
                           "k_tiled", "%d fixed 256-B keys" % n,
                           lambda p=[(keys, out)]: verify_fixed(p, 256, VERIFY_SAMPLES, 14),
                           grid_threads("fixed256", n)))
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
        vk = {"auto": 0, "span": 4, "span_pp": 6, "generic": 3, "round": 5}[args.var_kernel]
        wl.append(Workload("var", n, total / n + 8 + 16,
                           [lambda d=data, o=off, out=out, vk=vk, tb=total: hb.hash_var(d, o, out=out, kernel=vk, key_bytes=tb)],
                           {"generic": "k_generic", "round": "k_vround", "span": "k_span"}.get(args.var_kernel,
                                                                                               "k_span_pp"),
                           "%d variable keys U[8,512] B, %.3f GB of key bytes" % (n, total / 1e9),
                           lambda d=data, o=off, out=out: verify_var(d, o, out, VERIFY_SAMPLES, 15),
                           grid_threads("var", n) if args.var_kernel in ("auto", "span_pp") else None))
    for pname, tabs, dn in (("probe16", args.probe_tabs, 0), ("probe16_hbm", args.probe_tabs_hbm, 256)):
        if pname in only:
            wl.append(probe_workload(args, dev, pname, tabs, args.keys16 - dn, seed_base + (5 if dn == 0 else 8),
                                     bufs))
    if "tabpart" in only:
        wl.append(tab_workload(args, dev, seed_base))
    if "winorder" in only:
        wl.append(win_order_workload(args, dev, seed_base))
    if "hashwin16" in only:
        wl.append(hash_win_workload(args, dev, fixed16_pairs()))
    wl += ceiling_workloads(args, dev, only, bufs, fixed16_pairs)
    torch.cuda.synchronize()
    return sorted(wl, key=lambda w: ORDER.index(w.name) if w.name in ORDER else len(ORDER))


def probe_workload(args, dev, name, tabs, n, seed, bufs):
    """Row pre-probe: hash + row scan of every key against an
    index holding all of them (a get-hit batch), `tabs` physical tabs per window.
    Bytes per key: 16 key + 128 row + 16 record (+ the 2 MiB tab map once per
    launch). probe16 (16 tabs: 256 MiB of rows, the size of the Infinity Cache)
    is the cache-resident case; probe16_hbm (128 tabs: 2 GiB of rows) the HBM
    regime. unique_bytes counts each distinct row once (keys + distinct rows +
    records): the bytes HBM must deliver at least. probe16_hbm runs 256 keys
    fewer, so its launch grid (which the PMC rows are matched on) differs."""
    import torch

    import sharedhashfile_amd as hb
    from sharedhashfile_amd.keygen import device_random_bytes
    from sharedhashfile_amd.rowindex import synthetic_index

    keys = device_random_bytes(n * 16, seed, dev)
    h = hb.hash_fixed(keys, 16)
    tab_slot, rows, n_slots, placed = synthetic_index(h, tabs_per_win=tabs)
    index = hb.RowIndex(n_slots, tab_slot, rows)
    host_index = (tab_slot.cpu().numpy().view(np.uint32), rows.cpu().numpy(), n_slots)
    # each key's row (slot * 512 + row) in key order: the probe's own row sequence, for its ceiling
    h1 = h[:, 0]
    rid = (((h1 & 0xFF) * tabs + ((h1 >> 16) & 0x7FF) % tabs) * 512 + ((h1 >> 32) & 0x1FF)).to(torch.int32)
    distinct_rows = int(torch.unique(rid).numel())
    bufs[name + "_rows"] = (rows, rid, n)
    del h, tab_slot, h1
    out = torch.empty((n, 4), dtype=torch.int32, device=dev)

    def verify_probe(keys=keys, out=out, hx=host_index):
        import torch as _t

        from oracle.oracle_py import Oracle

        o = Oracle()
        idx = _sample_idx(n, VERIFY_SAMPLES, 16)
        ti = _t.from_numpy(idx).to(dev)
        k = keys.view(n, 16).index_select(0, ti).cpu().numpy()
        want = o.probe(o.hash_fixed(k, 16), hx[0], hx[1], hx[2])
        got = out.index_select(0, ti).cpu().numpy().view(np.uint32)
        return bool(np.array_equal(got, want)), int(idx.size)

    w = Workload(name, n, 16 + 128 + 16 + 4 * 256 * 2048 / n,
                 [lambda k=keys, o=out, ix=index: hb.probe_fixed(ix, k, 16, out=o)],
                 "k_fixed16<kOutProbe>", "%d fixed 16-B keys hashed and probed against a row index of "
                 "%d slots (%.0f MiB, %s) holding %d of them; %d distinct rows"
                 % (n, n_slots, n_slots / 16, "cache-resident" if n_slots * 65536 <= 256 << 20 else "HBM regime",
                    placed, distinct_rows), verify_probe, grid_threads(name, n))
    w.unique_bytes = 32.0 * n + 128.0 * distinct_rows
    bufs[name + "_unique"] = w.unique_bytes
    w.index = index
    return w


def ceiling_workloads(args, dev, only, bufs, fixed16_pairs):
    """The on-box ceilings (include/shf_hash_batch_ceiling.h), each on the
    buffers of the hashing line it bounds. `n` counts lanes; bytes_per_key is
    what one lane moves."""
    import torch

    import sharedhashfile_amd as hb
    from sharedhashfile_amd import bench_ceiling as bc

    wl = []
    if "ceil_copy" in only or "ceil_copy_hot" in only:
        pairs = fixed16_pairs()
        n = args.keys16
        if "ceil_copy" in only:
            wl.append(Workload("ceil_copy", n, 32,
                               [ceil_launcher(hb, bc.CEIL_COPY, k.data_ptr(), 16 * n, None, o.data_ptr(), n, dev)
                                for k, o in pairs], "k_ceil_copy",
                               "16-B/lane copy in k_fixed16's shape over fixed16's %d rotating batches" % len(pairs),
                               grid=grid_threads("ceil_copy", n)))
        if "ceil_copy_hot" in only:
            k, o = pairs[0]
            wl.append(Workload("ceil_copy_hot", n, 32,
                               [ceil_launcher(hb, bc.CEIL_COPY, k.data_ptr(), 16 * n, None, o.data_ptr(), n, dev)],
                               "k_ceil_copy", "the same copy over fixed16_hot's single batch",
                               grid=grid_threads("ceil_copy_hot", n)))
    if "ceil_copynt" in only or "ceil_copynt_hot" in only:
        pairs = fixed16_pairs()
        n = args.keys16
        if "ceil_copynt" in only:
            wl.append(Workload("ceil_copynt", n, 32,
                               [ceil_launcher(hb, bc.CEIL_COPY_NT, k.data_ptr(), 16 * n, None, o.data_ptr(), n, dev)
                                for k, o in pairs], "k_ceil_copyv<1>",
                               "the same copy with nontemporal stores (the fastest of tools/copy_sweep.py's variants) "
                               "over fixed16's %d rotating batches" % len(pairs), grid=grid_threads("ceil_copynt", n)))
        if "ceil_copynt_hot" in only:
            k, o = pairs[0]
            wl.append(Workload("ceil_copynt_hot", n, 32,
                               [ceil_launcher(hb, bc.CEIL_COPY_NT, k.data_ptr(), 16 * n, None, o.data_ptr(), n, dev)],
                               "k_ceil_copyv<1>", "the same over fixed16_hot's single batch",
                               grid=grid_threads("ceil_copynt_hot", n)))
    for name, kind, kern in (("ceil_copy_1b", bc.CEIL_COPY, "k_ceil_copy"), ("ceil_copynt_1b", bc.CEIL_COPY_NT,
                                                                                "k_ceil_copyv<1>")):
        if name not in only:
            continue
        keys, out, n = bufs["shard1b"]
        wl.append(Workload(name, n, 32,
                           [ceil_launcher(hb, kind, keys.data_ptr(), 16 * n, None, out.data_ptr(), n, dev)],
                           kern, "the same copy over shard1b's %d keys + hashes" % n, grid=grid_threads(name, n)))
    for cname, pname in (("ceil_probe_rows", "probe16"), ("ceil_probe_rows_hbm", "probe16_hbm")):
        if cname not in only or pname + "_rows" not in bufs:
            continue
        rows, rid, n = bufs[pname + "_rows"]
        out = torch.empty((n, 2), dtype=torch.int64, device=dev)
        rid16 = torch.zeros((n, 4), dtype=torch.int32, device=dev)  # the row in the first word of a 16-B record
        rid16[:, 0] = rid
        wl.append(Workload(cname, n, 160,
                           [ceil_launcher(hb, bc.CEIL_PROBE_ROWS, rows.data_ptr(), rows.numel(), rid16.data_ptr(),
                                          out.data_ptr(), n, dev)], "k_ceil_gather128<true>",
                           "%s's own row reads without the hash: a 16-B record per lane naming its key's 128-B "
                           "row (slot and row, in key order), the row fetched 8 lanes per row, a 16-B nt store: the "
                           "probe's 160 B per key, %d lanes" % (pname, n), grid=grid_threads(cname, n)))
        wl[-1].keep = (rows, rid16, out)
        wl[-1].unique_bytes = bufs.get(pname + "_unique")
    if {"ceil_read16", "ceil_read16nt", "ceil_read16w1"} & set(only):
        n = read16_lanes(args, only)
        if "fixed256" in bufs:
            keys, out, _ = bufs["fixed256"]
            where = "fixed256's keys and hashes"
        else:
            keys = torch.empty(n * 256, dtype=torch.uint8, device=dev)
            out = torch.empty((n, 2), dtype=torch.int64, device=dev)
            where = "a buffer of its own"
        for name, kind, st in (("ceil_read16", bc.CEIL_READ16, "plain"), ("ceil_read16nt", bc.CEIL_READ16_NT, "nt"),
                               ("ceil_read16w1", bc.CEIL_READ16_W1, "nt, one wave per workgroup")):
            if name not in only:
                continue
            wl.append(Workload(name, n, 272,
                               [ceil_launcher(hb, kind, keys.data_ptr(), 256 * n, None, out.data_ptr(), n, dev)],
                               KERNEL_SYMS[name].rstrip("("),
                               "16:1 read-mostly copy (16 x 16 B nt loads per lane, one contiguous 16 KiB per wave, "
                               "16-B %s store) over %s, %d lanes" % (st, where, n), grid=grid_threads(name, n)))
            wl[-1].keep = (keys, out)
    if "ceil_gather128" in only:
        n = args.keys16
        rows = torch.empty(n * 128, dtype=torch.uint8, device=dev)
        idx = torch.randperm(n, device=dev, dtype=torch.int32)
        out = torch.empty((n, 2), dtype=torch.int64, device=dev)
        wl.append(Workload("ceil_gather128", n, 148,
                           [ceil_launcher(hb, bc.CEIL_GATHER128, rows.data_ptr(), rows.numel(), idx.data_ptr(),
                                          out.data_ptr(), n, dev)], "k_ceil_gather128",
                           "each of %d 128-B rows read once in random order, 8 lanes per row (the probe's row fetch) "
                           "+ 4-B index + 16-B store per lane" % n, grid=grid_threads("ceil_gather128", n)))
        wl[-1].keep = (rows, idx, out)
    if "ceil_stream16u" in only:
        n = 2 * args.keys16
        bs = [(torch.empty(16 * n + 16, dtype=torch.uint8, device=dev), torch.empty((n, 2), dtype=torch.int64,
                                                                                    device=dev)) for _ in range(2)]
        wl.append(Workload("ceil_stream16u", n, 32,
                           [ceil_launcher(hb, bc.CEIL_STREAM16U, s_.data_ptr(), s_.numel(), None, o.data_ptr(), n, dev)
                            for s_, o in bs], "k_ceil_stream16u",
                           "16-B loads 7 bytes off alignment (the tab copy's record loads) + 16-B stores, %d lanes, "
                           "2 rotating buffers" % n, grid=grid_threads("ceil_stream16u", n)))
        wl[-1].keep = bs
    for name, kind in (("ceil_valu_add", bc.CEIL_VALU_ADD), ("ceil_valu_mul", bc.CEIL_VALU_MUL)):
        if name not in only:
            continue
        out = torch.empty((VALU_LANES, 2), dtype=torch.int64, device=dev)
        w = Workload(name, VALU_LANES, 16, [ceil_launcher(hb, kind, 1, VALU_ITERS, None, out.data_ptr(), VALU_LANES,
                                                          dev)], "k_ceil_valu",
                     "VALU-saturating launch: 8 independent %s chains x %d rounds per lane, %d lanes (32 waves/CU)"
                     % ("v_add_u32" if kind == bc.CEIL_VALU_ADD else "v_mul_lo_u32", VALU_ITERS, VALU_LANES),
                     grid=grid_threads(name, VALU_LANES))
        w.unit = "VALU lane-ops/s"
        w.ops_per_key = 8 * VALU_ITERS
        w.keep = out
        wl.append(w)
    for w in wl:
        if not hasattr(w, "unit"):
            w.unit = "lanes/s"
    return wl


def win_order_workload(args, dev, seed_base):
    """Window order (SURVEY.md §8 f1's use; shf_win_order_async): the key
    indices of 10M hash records stably sorted by h1 & 0xff. Algorithmic bytes
    per key: the 16-B record read once + the 4-B index written (20 B); the
    library's passes add one window byte written and read per key."""
    import ctypes

    import torch

    import sharedhashfile_amd as hb
    from sharedhashfile_amd.keygen import device_random_bytes

    n = args.keys16
    hashes = device_random_bytes(n * 16, seed_base + 7, dev).view(torch.int64).view(n, 2)
    perm = torch.empty(n, dtype=torch.int32, device=dev)
    start = torch.empty(257, dtype=torch.int32, device=dev)
    lib = hb.load()
    ws = torch.empty(lib.shf_win_order_workspace_bytes(n), dtype=torch.uint8, device=dev)
    fn = lib.shf_win_order_async
    argv = (ctypes.c_void_p(hashes.data_ptr()), ctypes.c_uint64(n), ctypes.c_void_p(perm.data_ptr()),
            ctypes.c_void_p(start.data_ptr()), ctypes.c_void_p(ws.data_ptr()), ctypes.c_size_t(ws.numel()),
            ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream))

    def launch():
        rc = fn(*argv)
        if rc:
            raise hb.ShfHashBatchError(rc, "shf_win_order_async")

    def verify():
        from oracle.oracle_py import Oracle

        want_p, want_s = Oracle.win_order(hashes.cpu().numpy().view(np.uint64))
        ok = (np.array_equal(perm.cpu().numpy().view(np.uint32), want_p) and
              np.array_equal(start.cpu().numpy().view(np.uint32), want_s))
        return bool(ok), int(n)

    return Workload("winorder", n, 16 + 4, [launch], "k_wo_rank + k_wo_scan_rows + k_wo_place",
                    "%d 16-B hash records ordered by window (stable counting sort, 3 launches)" % n, verify,
                    grid_threads("winorder", n))


def hash_win_workload(args, dev, pairs):
    """Hash + window order in one call (shf_hash_batch_fixed_win_async, SURVEY.md
    §8 f1 "alongside"): configs[1]'s 10M 16-B keys -> 16-B records + the window
    order (perm, win_start), rotating over fixed16's batches with an order buffer
    and workspace each. Algorithmic bytes per key: 16 key + 16 record + 4 perm."""
    import ctypes

    import torch

    import sharedhashfile_amd as hb

    n = args.keys16
    lib = hb.load()
    need = lib.shf_win_order_workspace_bytes(n)
    fn = lib.shf_hash_batch_fixed_win_async
    st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    bufs, launches = [], []
    for keys, out in pairs:
        perm = torch.empty(n, dtype=torch.int32, device=dev)
        start = torch.empty(257, dtype=torch.int32, device=dev)
        ws = torch.empty(need, dtype=torch.uint8, device=dev)
        bufs.append((keys, out, perm, start, ws))
        argv = (ctypes.c_void_p(keys.data_ptr()), ctypes.c_uint32(16), ctypes.c_uint64(n), ctypes.c_uint32(SEED),
                ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(perm.data_ptr()), ctypes.c_void_p(start.data_ptr()),
                ctypes.c_void_p(ws.data_ptr()), ctypes.c_size_t(need), st)

        def launch(argv=argv):
            rc = fn(*argv)
            if rc:
                raise hb.ShfHashBatchError(rc, "shf_hash_batch_fixed_win_async")

        launches.append(launch)

    def verify():
        from oracle.oracle_py import Oracle

        ok, checked = verify_fixed([(b[0], b[1]) for b in bufs], 16, VERIFY_SAMPLES, 17)
        for keys, out, perm, start, _ in bufs[:1]:  # the whole order of one batch, from its own records
            want_p, want_s = Oracle.win_order(out.cpu().numpy().view(np.uint64))
            ok = ok and np.array_equal(perm.cpu().numpy().view(np.uint32), want_p) and \
                np.array_equal(start.cpu().numpy().view(np.uint32), want_s)
            checked += n
        return bool(ok), int(checked)

    w = Workload("hashwin16", n, 16 + 16 + 4, launches, "k_fixed16_win + k_wo_scan_rows + k_wo_place",
                 "%d 16-B keys hashed and window-ordered in one call (records + perm), rotating over %d batches"
                 % (n, len(pairs)), verify, grid_threads("hashwin16", n))
    w.keep = bufs
    return w


def tab_workload(args, dev, seed_base):
    """f4: shf_tab_part()'s copy of a batch of full tabs,
    one job per tab (shf.c:722-779 + the shrink :678-720), device-resident.
    Synthetic tabs at part time (sharedhashfile_amd/tabgen.py: 4500 refs,
    keys U[16,64] B, values U[8,128] B, ~0.5 MB of records each), every job
    its own copy in HBM so that nothing is re-read from cache."""
    import ctypes

    import torch

    import sharedhashfile_amd as hb
    from sharedhashfile_amd.tabgen import algorithmic_bytes, synth_tab

    nb = 8
    base = [synth_tab(seed_base + 50 + i) for i in range(nb)]
    maps, news = [], []
    for _, m, old in base:
        new = (old + 1000) % 2048
        maps.append(hb.tab_part_redirect(m, old, new))
        news.append(new)
    al = lambda x: (x + 4095) // 4096 * 4096
    J = args.tab_jobs
    sizes = [al(img.size) for img, _, _ in base]
    jobs = (hb.TabJob * J)()
    soff = doff = 0
    for j in range(J):
        b = j % nb
        jb = jobs[j]
        jb.src, jb.src_len, jb.cap, jb.map, jb.tab_new = soff, base[b][0].size, sizes[b], b, news[b]
        jb.keep, jb.move = doff, doff + sizes[b]
        jb.keep_type, jb.move_type = 0x3E, 0x3E
        soff += sizes[b]
        doff += 2 * sizes[b]
    src = torch.zeros(soff, dtype=torch.uint8, device=dev)
    for b, (img, _, _) in enumerate(base):
        t = torch.from_numpy(img).to(dev)
        for j in range(b, J, nb):
            src[jobs[j].src:jobs[j].src + img.size].copy_(t)
    dst = torch.zeros(doff, dtype=torch.uint8, device=dev)
    d_jobs = torch.from_numpy(np.frombuffer(bytes(jobs), dtype=np.uint8).copy()).to(dev)
    d_maps = torch.from_numpy(np.stack(maps).view(np.int16)).to(dev)
    prm = hb.TabParams(0, 0, 0, 1)
    fn = hb.load().shf_tab_copy_batch_async
    argv = (ctypes.c_void_p(src.data_ptr()), ctypes.c_uint64(soff), ctypes.c_void_p(dst.data_ptr()),
            ctypes.c_uint64(doff), ctypes.c_void_p(d_jobs.data_ptr()), ctypes.c_uint32(J),
            ctypes.c_void_p(d_maps.data_ptr()), ctypes.c_uint32(nb), ctypes.byref(prm),
            ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream))

    def launch():
        rc = fn(*argv)
        if rc:
            raise hb.ShfHashBatchError(rc, "shf_tab_copy_batch_async")

    def verify():
        from oracle.oracle_py import Oracle

        o = Oracle()
        done = (hb.TabJob * J).from_buffer_copy(d_jobs.cpu().numpy().tobytes())
        if any(done[j].status != hb.OK for j in range(J)):
            return False, 0
        ok, checked = True, 0
        for j in sorted({0, J - 1, J // 3, (2 * J) // 3} | set(range(min(nb, J)))):
            b = j % nb
            keep = dst[jobs[j].keep:jobs[j].keep + sizes[b]].cpu().numpy()
            move = dst[jobs[j].move:jobs[j].move + sizes[b]].cpu().numpy()
            wk, wm = o.tab_split(base[b][0], maps[b], news[b], cap=sizes[b], keep_type=0x3E, move_type=0x3E)
            ok = ok and np.array_equal(keep, wk) and np.array_equal(move, wm)
            checked += 1
        return bool(ok), checked

    per_job = float(np.mean([algorithmic_bytes(base[j % nb][0]) for j in range(J)]))
    w = Workload("tabpart", J, per_job, [launch], "k_tab_split",
                 "%d tab parts per step (f4: shf_tab_part's copy, both output tabs), synthetic tabs of 4500 refs "
                 "with %.2f MB of records each, %.2f GB moved per step" % (
                     J, float(np.mean([img.size - 65560 for img, _, _ in base])) / 1e6, J * per_job / 1e9), verify,
                 grid_threads("tabpart", J))
    w.unit = "tabs/s"
    w.keep = (src, dst, d_jobs, d_maps, prm)
    return w


def time_workload(w, steps, warmup, repeats, dist, dist_dev, warmup_min_s=WARMUP_MIN_S):
    """Per repeat: (wall seconds for `steps` steps, max over ranks; mean per-launch
    device seconds from HIP events on the launch stream, max over ranks; the
    same, this rank's own)."""
    import torch

    stream = torch.cuda.current_stream()  # the stream every launch goes to (hb passes it to the library)
    # W warmup steps, continued (untimed) until the GPU has run this workload
    # for warmup_min_s: after seconds of host-side setup the clocks start low,
    # and 10 steps of a 50-us kernel are not enough to bring them up.
    t_w = time.perf_counter()
    done = 0
    while done < warmup or time.perf_counter() - t_w < warmup_min_s:
        w.launch(done)
        done += 1
        if done >= warmup and done % 16 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    walls, devs, enq = [], [], []
    for _ in range(repeats):
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev0.record(stream)
        for i in range(steps):
            w.launch(i)
        ev1.record(stream)
        t_enq = time.perf_counter()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        if dist:
            dist.barrier()
        walls.append(t1 - t0)
        # HIP events bracketing the timed region on the launch stream: mean device
        # time per launch, back-to-back kernels (inter-kernel gaps included)
        devs.append(ev0.elapsed_time(ev1) / steps / 1e3)
        enq.append(t_enq - t0)
    devs_local = list(devs)
    if dist:
        import torch as _t

        t = _t.tensor(walls + devs, dtype=_t.float64, device=dist_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        walls, devs = [float(x) for x in t[:repeats]], [float(x) for x in t[repeats:]]
    w.enqueue_s = float(np.median(enq))
    return walls, devs, devs_local


# ---------------------------------------------------------------------------
# host-inclusive rate: keys start and hashes end in host memory
# ---------------------------------------------------------------------------
PCIE_MB = 160  # bytes per direction of the PCIe ceiling copies


def pcie_ceilings(dev, mb=PCIE_MB, reps=5):
    """The PCIe ceiling of this box, measured in the same run as the host lines
    it bounds, by the two mechanisms the host pipelines use:
      * the copy engines: hipMemcpyAsync (torch copy_, non_blocking) of `mb` MB
        between page-locked host memory and HBM, host -> device alone (h2d),
        device -> host alone (d2h), and both at once on two streams (both: the
        two directions' bytes over the later finish; both_h2d / both_d2h: each
        direction timed by HIP events on its own stream);
      * a kernel over PCIe (zero copy): the bench library's 16-B copy kernel
        (SHF_HB_CEIL_COPY, k_fixed16's access shape) reading page-locked host
        memory into HBM (zc_h2d), HBM into host memory (zc_d2h), and host into
        host (zc_both: `mb` MB each way at once);
    plus the HIP runtime's own pageable host -> device copy (h2d_pageable: the
    path pageable fixed-length keys take). GB/s (1e9 B/s), median of `reps`
    after one untimed run of each."""
    import torch

    nb = mb * 1_000_000
    h_src = torch.empty(nb, dtype=torch.uint8).pin_memory()
    h_dst = torch.empty(nb, dtype=torch.uint8).pin_memory()
    h_pg = torch.from_numpy(np.ones(nb, dtype=np.uint8))  # pageable
    d_a = torch.empty(nb, dtype=torch.uint8, device=dev)
    d_b = torch.empty(nb, dtype=torch.uint8, device=dev)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def one(copies):  # copies: [(stream, dst, src)] started together; ms per copy, on its own stream
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in copies]
        torch.cuda.synchronize(dev)
        for (st, dst, src), (a, b) in zip(copies, evs):
            with torch.cuda.stream(st):
                a.record(st)
                dst.copy_(src, non_blocking=True)
                b.record(st)
        torch.cuda.synchronize(dev)
        return [a.elapsed_time(b) for a, b in evs]

    def med(copies):
        one(copies)
        runs = [one(copies) for _ in range(reps)]
        return [float(np.median([r[i] for r in runs])) for i in range(len(copies))]

    from sharedhashfile_amd import bench_ceiling as bc

    zc_src, zc_dst = bc.host_device_ptr(h_src.data_ptr()), bc.host_device_ptr(h_dst.data_ptr())
    copy_fn = bc.load().shf_hb_ceiling_async

    def zc(src, dst):  # ms of one 16-B-per-lane copy kernel, nb bytes read and nb written
        st = torch.cuda.current_stream(dev)
        ts = []
        for r in range(reps + 1):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize(dev)
            a.record(st)
            rc = copy_fn(bc.CEIL_COPY, ctypes.c_void_p(src), nb, None, ctypes.c_void_p(dst), nb // 16,
                         ctypes.c_void_p(st.cuda_stream))
            b.record(st)
            torch.cuda.synchronize(dev)
            if rc:
                raise RuntimeError("shf_hb_ceiling_async over PCIe: %d" % rc)
            if r:
                ts.append(a.elapsed_time(b))
        return float(np.median(ts))

    gbs = lambda ms: nb / (ms * 1e-3) / 1e9  # noqa: E731
    zc_h2d, zc_d2h, zc_both = zc(zc_src, d_a.data_ptr()), zc(d_b.data_ptr(), zc_dst), zc(zc_src, zc_dst)
    h2d, = med([(s1, d_a, h_src)])
    d2h, = med([(s2, h_dst, d_b)])
    both_h2d, both_d2h = med([(s1, d_a, h_src), (s2, h_dst, d_b)])
    pg = []
    for _ in range(reps + 1):  # the runtime's pageable copy holds the calling thread: wall clock
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        d_a.copy_(h_pg)
        torch.cuda.synchronize(dev)
        pg.append(time.perf_counter() - t0)
    return {"h2d": round(gbs(h2d), 2), "d2h": round(gbs(d2h), 2),
            "both_h2d": round(gbs(both_h2d), 2), "both_d2h": round(gbs(both_d2h), 2),
            "both": round(2 * nb / (max(both_h2d, both_d2h) * 1e-3) / 1e9, 2),
            "h2d_pageable": round(nb / float(np.median(pg[1:])) / 1e9, 2),
            "zc_h2d": round(gbs(zc_h2d), 2), "zc_d2h": round(gbs(zc_d2h), 2), "zc_both": round(2 * gbs(zc_both), 2),
            "bytes_per_copy": nb}


def pcie_bound(ceil, bytes_in, bytes_out):
    """Keys/s the PCIe ceilings allow a line moving bytes_in host -> device and
    bytes_out device -> host per key, by the better of the two mechanisms
    (copy engines, or a kernel over PCIe: keys "zc_*"): through one, no faster
    than either direction alone, nor than both directions' aggregate when they
    run at once."""
    best = 0.0
    for pre in ("", "zc_"):
        if pre + "h2d" not in ceil:
            continue
        t = max(bytes_in / (ceil[pre + "h2d"] * 1e9), bytes_out / (ceil[pre + "d2h"] * 1e9),
                (bytes_in + bytes_out) / (ceil[pre + "both"] * 1e9))
        best = max(best, 1.0 / t)
    return best


def time_host_inclusive(args, dev):
    """Host buffers in and out (SHF_HASH_MEM_HOST): H2D keys (+ offsets) +
    kernel + D2H hashes, pipelined in SHF_HB_STAGE_MB chunks, SHF_HB_SLOTS in
    flight. Pageable fixed-length keys go through the HIP runtime's pageable
    copy with the records copied out on the library's copy threads beside it,
    pageable variable-length keys are staged through pinned memory on the CPU;
    page-locked buffers are DMA'd directly. Fixed 16-B keys and config-D's U[8,512] B
    variable-length keys, --host-keys of each."""
    import torch

    import sharedhashfile_amd as hb
    from sharedhashfile_amd.keygen import device_random_bytes

    lib = hb.load()
    n = args.host_keys
    res = {"unit": "keys/s", "note": "never `value`: PCIe-bound; sample = %d keys per batch, median of the "
                                     "timed repeats after two untimed calls; *_pinned = page-locked caller buffers "
                                     "(16-B keys: the kernel reads and writes them over PCIe, zero copy), "
                                     "*_pinned_staged = the same through hipMemcpyAsync both ways; "
                                     "*_pageable = pageable buffers through the pipeline (fixed-length keys by the "
                                     "runtime's pageable copy, variable-length ones staged on the CPU; the library "
                                     "never page-locks a caller's pageable memory); *_x16 = 16 threads, one slice each, "
                                     "at once (one staging pool); uid16_* = 8-B UID parts back instead of 16-B hashes "
                                     "(shf_uid_parts_batch_fixed). Per line: wire_bytes per key (in + out over PCIe), "
                                     "pcie_bound = keys/s the same run's PCIe ceilings allow those bytes "
                                     "(bench.py pcie_bound), frac_of_pcie = value / pcie_bound"
                                     % n}
    ceil = pcie_ceilings(dev)
    res["ceilings_gbs"] = ceil

    def _staged(fn, var="SHF_HB_ZERO_COPY_MAX_KEY"):  # through the copy-engine pipeline (zero copy off)
        old = os.environ.get(var)
        os.environ[var] = "0"
        try:
            return fn()
        finally:
            if old is None:
                os.environ.pop(var, None)
            else:
                os.environ[var] = old
    def _threaded(k, call):  # k threads over even slices of [0, n); the first failing status, else 0
        import threading

        rcs = [0] * k
        ts = [threading.Thread(target=lambda i=i: rcs.__setitem__(i, call(n * i // k, n * (i + 1) // k)))
              for i in range(k)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        return next((r for r in rcs if r), 0)
    keys = device_random_bytes(n * 16, 77, dev).cpu().numpy()
    g = torch.Generator(device=dev)
    g.manual_seed(78)
    lens = torch.randint(8, 513, (n,), generator=g, device=dev, dtype=torch.int64)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens.cpu().numpy())
    data = device_random_bytes(int(off[-1]), 79, dev).cpu().numpy()
    del lens
    pk = torch.from_numpy(keys).pin_memory()
    po = torch.empty((n, 2), dtype=torch.int64).pin_memory()
    out = np.empty((n, 2), dtype=np.uint64)
    pd = torch.from_numpy(data).pin_memory()
    poff = torch.from_numpy(off.view(np.int64)).pin_memory()
    vout = np.empty((n, 2), dtype=np.uint64)
    vpo = torch.empty((n, 2), dtype=torch.int64).pin_memory()
    uout = np.empty(n, dtype=np.uint64)
    upo = torch.empty(n, dtype=torch.int64).pin_memory()
    perm = np.empty(n, dtype=np.uint32)
    cases = [
        ("fixed16_pageable", lambda: lib.shf_hash_batch_fixed(keys.ctypes.data, 16, n, SEED, out.ctypes.data,
                                                              hb.MEM_HOST), 5),
        ("fixed16_pinned", lambda: lib.shf_hash_batch_fixed(pk.data_ptr(), 16, n, SEED, po.data_ptr(), hb.MEM_HOST),
         5),
        ("fixed16_pinned_staged", lambda: _staged(lambda: lib.shf_hash_batch_fixed(pk.data_ptr(), 16, n, SEED,
                                                                                   po.data_ptr(), hb.MEM_HOST)), 5),
        ("var_pageable", lambda: lib.shf_hash_batch_var(data.ctypes.data, off.ctypes.data, n, SEED, vout.ctypes.data,
                                                        hb.MEM_HOST), 3),
        ("var_pinned", lambda: lib.shf_hash_batch_var(pd.data_ptr(), poff.data_ptr(), n, SEED, vpo.data_ptr(),
                                                      hb.MEM_HOST), 3),
        # the reference's usage model, many threads of one process (test.f.shf.c:274-336): 16 threads each
        # hash a 1/16 slice of the same pageable batch at once, sharing the one staging pool
        ("fixed16_pageable_x16", lambda: _threaded(16, lambda lo, hi: lib.shf_hash_batch_fixed(
            keys.ctypes.data + lo * 16, 16, hi - lo, SEED, out.ctypes.data + lo * 16, hb.MEM_HOST)), 5),
        # 8-B UID parts (the bits shf.c:800-803 reads) back instead of the 16-B hash
        ("uid16_pageable", lambda: lib.shf_uid_parts_batch_fixed(keys.ctypes.data, 16, n, SEED, uout.ctypes.data,
                                                                 hb.MEM_HOST), 5),
        ("uid16_pinned", lambda: lib.shf_uid_parts_batch_fixed(pk.data_ptr(), 16, n, SEED, upo.data_ptr(),
                                                               hb.MEM_HOST), 5),
        ("uid16_pinned_staged", lambda: _staged(lambda: lib.shf_uid_parts_batch_fixed(pk.data_ptr(), 16, n, SEED,
                                                                                      upo.data_ptr(), hb.MEM_HOST)),
         5),
        # hash (or UID parts) + window order in one call: the order (4 B/key) comes back too
        # (shf_put_batch_var_win_ordered / _parts_win_ordered's GPU call)
        ("hashwin16_pageable", lambda: lib.shf_hash_batch_fixed_win(keys.ctypes.data, 16, n, SEED, out.ctypes.data,
                                                                    perm.ctypes.data, None, hb.MEM_HOST), 5),
        ("uidwin16_pageable", lambda: lib.shf_uid_parts_batch_fixed_win(keys.ctypes.data, 16, n, SEED,
                                                                        uout.ctypes.data, perm.ctypes.data, None,
                                                                        hb.MEM_HOST), 5),
    ]
    mean_len = float(off[-1]) / n
    wire = {"fixed16": (16, 16), "var": (mean_len + 8, 16), "uid16": (16, 8), "hashwin16": (16, 20),
            "uidwin16": (16, 12)}  # (host->device, device->host) B/key
    for name, fn, reps in cases:
        # two untimed calls: the HIP runtime's first hipMemcpyAsync calls from a page-locked buffer it has not
        # copied from before take 7-14 ms to enqueue instead of 0.03 ms (SHF_HB_TRACE copy_in_ms, round 6:
        # profiles/r6/host_uid/), which made single slow repeats of *_pinned_staged (0.85-0.92 G keys/s);
        # their times are kept in untimed_ms
        untimed = []
        for _ in range(2):
            t0 = time.perf_counter()
            rc = fn()
            untimed.append(round((time.perf_counter() - t0) * 1e3, 3))
            if rc:
                raise hb.ShfHashBatchError(rc, "host-inclusive " + name)
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            rc = fn()
            ts.append(time.perf_counter() - t0)
            if rc:
                raise hb.ShfHashBatchError(rc, "host-inclusive " + name)
        res[name] = {"value": n / float(np.median(ts)), "value_min": n / max(ts), "value_max": n / min(ts),
                     "repeats": reps, "untimed_ms": untimed}
        b_in, b_out = wire[name.split("_")[0]]
        bound = pcie_bound(ceil, b_in, b_out)
        res[name].update({"wire_bytes": round(b_in + b_out, 1), "pcie_bound": bound,
                          "frac_of_pcie": round(res[name]["value"] / bound, 3)})
    # sampled check of the host outputs (the oracle is the checker)
    try:
        from oracle.oracle_py import Oracle

        o = Oracle()
        idx = _sample_idx(n, VERIFY_SAMPLES, 21)
        want = o.hash_fixed(keys.reshape(n, 16)[idx], 16)
        ok = np.array_equal(out[idx], want) and np.array_equal(po.numpy().view(np.uint64)[idx], want)
        sub_lens = (off[idx + 1] - off[idx]).astype(np.int64)
        sub = np.concatenate([data[int(off[i]):int(off[i + 1])] for i in idx])
        so = np.zeros(idx.size + 1, dtype=np.uint64)
        so[1:] = np.cumsum(sub_lens)
        vw = o.hash_var(sub, so)
        ok = ok and np.array_equal(vout[idx], vw) and np.array_equal(vpo.numpy().view(np.uint64)[idx], vw)
        uw = o.uid_parts(want)
        ok = ok and np.array_equal(uout[idx], uw) and np.array_equal(upo.numpy().view(np.uint64)[idx], uw)
        # the window order of the last call (uidwin16): the stable order of every key's window byte
        ok = ok and np.array_equal(perm, np.argsort((uout & np.uint64(0xFF)).astype(np.int64), kind="stable"))
        res["verified"] = bool(ok)
    except Exception as e:  # noqa: BLE001
        res["verified"] = None
        res["verify_note"] = "oracle unavailable: %s" % e
    res["var_mean_key_bytes"] = float(off[-1]) / n
    return res


# ---------------------------------------------------------------------------
# CPU baseline: the reference's own shf_make_hash() loop (test.9 shape)
# ---------------------------------------------------------------------------
def host_cpus():
    """CPUs this process may run on: the affinity mask, capped by a cgroup v2
    cpu.max quota when there is one."""
    vis = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = vis
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
            if q != "max":
                quota = float(q) / float(period)
    except (OSError, ValueError):
        pass
    return {"visible": vis, "affinity": aff, "cgroup_quota_cpus": quota}


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

    fold = ctypes.c_uint64(0)
    o = None
    if ref is None:
        from oracle.oracle_py import Oracle

        o = Oracle()

    def run(passes, threads):
        if ref is not None:
            return ref.ref_bench_make_hash_loop(keys.ctypes.data, L, n, passes, threads, ctypes.byref(fold))
        t0 = time.perf_counter()
        for _ in range(passes):
            o.hash_fixed(keys, L, threads=threads)
        return time.perf_counter() - t0

    if ref is not None:
        kind, what = "reference", "oracle/_ref/libref_shf.so: reference src/shf.c shf_make_hash() + src/murmurhash3.c, gcc -O2"
    else:
        kind, what = "port", "oracle/murmur3_oracle.c restatement, gcc -O2"
    dt1 = run(1, 1)
    passes = max(1, int(args.cpu_seconds / max(dt1, 1e-6)))
    dt = run(passes, 1)
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            model = next((l.split(":", 1)[1].strip() for l in f if l.startswith("model name")), "")
    except OSError:
        pass
    cpus = host_cpus()
    one = n * passes / dt
    out = {"value": one, "unit": "keys/s", "cores": 1, "kind": kind,
           "sample": "%d passes x 1M 16-B keys (test.9 loop shape, hash only), %.1f s, one thread, %s; host %s"
                     % (passes, dt, what, model),
           "host_cpus": cpus}
    # SURVEY.md s8(d) config A also asks for the host's cores. This box's rule
    # sizes host worker pools to its CPU share per GPU (16 threads): that leg is
    # measured (the whole host's CPUs are not this job's to use).
    threads = min(BOX_CPU_SHARE, cpus["affinity"])
    if threads > 1:
        mt_passes = max(1, int(passes * threads / 4))  # ~1/4 of the single-thread time if it scales
        dt_mt = run(mt_passes, threads)
        v = n * mt_passes / dt_mt
        out["threads%d" % threads] = {"value": v, "unit": "keys/s", "cores": threads,
                                      "sample": "%d passes x 1M 16-B keys over %d threads (even key ranges), %.1f s"
                                                % (mt_passes, threads, dt_mt)}
    return out


# ---------------------------------------------------------------------------
# rocprofv3 PMC passes (child processes, N=1 only): HBM bytes, VALU, waits
# ---------------------------------------------------------------------------
RDREQ = ["TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum", "TCC_EA0_RDREQ_sum"]
PMC_PASSES = [["FETCH_SIZE"], ["WRITE_SIZE"], RDREQ,
              ["SQ_ACTIVE_INST_VALU", "SQ_INSTS_VALU", "SQ_WAVES", "SQ_WAIT_ANY", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES",
               "GRBM_GUI_ACTIVE"]]
PMC_SKIP = ("fixed16_hot", "shard1b", "ceil_copy_hot", "ceil_copy_1b", "ceil_copynt_hot", "ceil_copynt_1b",
            "ceil_probe_rows", "ceil_probe_rows_hbm")  # same kernels and grids as measured ones


def pmc_child_sizes(args, want):
    """Lanes / keys / jobs of each workload in the PMC child (configs 2 and 3
    at <= 10M keys: their per-key figures do not depend on the batch size)."""
    k256, kvar = min(args.keys256, 10_000_000), min(args.keysvar, 10_000_000)
    child = argparse.Namespace(keys256=k256, keys16=args.keys16)
    sizes = {"fixed16": args.keys16, "fixed256": k256, "var": kvar, "probe16": args.keys16,
             "probe16_hbm": args.keys16 - 256,
             "tabpart": args.tab_jobs, "winorder": args.keys16, "hashwin16": args.keys16, "ceil_copy": args.keys16, "ceil_copynt": args.keys16,
             "ceil_read16": read16_lanes(child, set(want)), "ceil_read16nt": read16_lanes(child, set(want)),
             "ceil_read16w1": read16_lanes(child, set(want)),
             "ceil_gather128": args.keys16, "ceil_stream16u": 2 * args.keys16, "ceil_valu_add": VALU_LANES,
             "ceil_valu_mul": VALU_LANES}
    return {w: sizes[w] for w in want if w in sizes}, k256, kvar


def parse_pmc_rows(rows, grids):
    """{workload: {counter: [values]}} from rocprofv3 counter_collection rows:
    a row counts for a workload when its kernel name holds the workload's
    symbol and its grid is the workload's launch grid. A kernel that several
    multi-kernel workloads share (MULTI_KERNEL: the order passes) counts for the
    workload whose own first kernel ran last before it (rows in dispatch order)."""
    vals = {}
    multi = [w for w in grids if w in MULTI_KERNEL]
    owner_of = {}  # a multi-kernel workload's own kernels (those no other workload of the run has)
    for w in multi:
        for sym in MULTI_KERNEL[w]:
            if sum(sym in MULTI_KERNEL[v] for v in multi) == 1:
                owner_of[sym] = w

    def order(r):
        try:
            return int(float(r.get("Dispatch_Id") or 0))
        except ValueError:
            return 0
    current = None
    for row in sorted(rows, key=order):
        name = row.get("Kernel_Name", "")
        try:
            grid = int(float(row.get("Grid_Size") or -1))
        except ValueError:
            grid = -1
        own = next((w for sym, w in owner_of.items() if sym in name), None)
        if own is not None:
            current = own
        for w, g in grids.items():
            if w in MULTI_KERNEL:
                for sym in MULTI_KERNEL[w]:
                    if sym in name and (own == w or (own is None and (sym in owner_of or current == w))):
                        vals.setdefault(w, {}).setdefault((sym, row.get("Counter_Name")), []).append(
                            float(row["Counter_Value"]))
            elif KERNEL_SYMS[w] in name and (g is None or grid < 0 or grid == g):
                vals.setdefault(w, {}).setdefault(row.get("Counter_Name"), []).append(float(row["Counter_Value"]))
    return vals


def pmc_medians(cs):
    """{counter: median per launch} of one workload's rows; a multi-kernel
    workload's counters are the sum of its kernels' medians."""
    out = {}
    for c, v in cs.items():
        if isinstance(c, tuple):
            out[c[1]] = out.get(c[1], 0.0) + float(np.median(v))
        else:
            out[c] = float(np.median(v))
    return out


def collect_pmc(args, names):
    """One rocprofv3 --pmc pass per counter group over a short child bench of
    the given workloads. Returns ({workload: {counter: median per launch,
    "_lanes": n in the child}}, note)."""
    prof = shutil.which("rocprofv3")
    if not prof:
        return None, "rocprofv3 not found"
    want = [x for x in names if x in KERNEL_SYMS and x not in PMC_SKIP]
    sizes, k256, kvar = pmc_child_sizes(args, want)
    grids = {w: grid_threads(w, sizes[w]) for w in want}
    if args.var_kernel not in ("auto", "span_pp"):
        grids.pop("var", None)
        want = [w for w in want if w != "var"]
    res = {w: {"_lanes": sizes[w]} for w in want}
    for group in PMC_PASSES:
        outdir = tempfile.mkdtemp(prefix="shfhb_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
        cmd = [prof, "--pmc"] + group + ["--output-format", "csv", "-d", outdir, "-o", "pmc", "--",
                                         sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup",
                                         "1", "--repeats", "1", "--only", ",".join(want), "--no-cpu", "--no-verify",
                                         "--no-host-inclusive", "--traffic", "off", "--quiet", "--keys16",
                                         str(args.keys16), "--keys256", str(k256), "--keysvar", str(kvar),
                                         "--tab-jobs", str(args.tab_jobs), "--warmup-min-s", "0", "--gpus", "1",
                                         "--probe-tabs", str(args.probe_tabs), "--probe-tabs-hbm",
                                         str(args.probe_tabs_hbm),
                                         "--fixed-kernel", args.fixed_kernel, "--var-kernel", args.var_kernel]
        try:
            subprocess.run(cmd, check=True, timeout=300, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                           cwd=os.environ.get("TMPDIR", "/tmp"))
        except Exception as e:  # noqa: BLE001
            shutil.rmtree(outdir, ignore_errors=True)
            return None, "rocprofv3 --pmc %s failed: %s" % (" ".join(group), e)
        rows = []
        for f in glob.glob(os.path.join(outdir, "**", "*counter_collection*.csv"), recursive=True):
            with open(f) as fh:
                rows += list(csv.DictReader(fh))
        shutil.rmtree(outdir, ignore_errors=True)
        for w, cs in parse_pmc_rows(rows, grids).items():
            res[w].update(pmc_medians(cs))
    return res, ("per launch, median over the child's launches of each workload's kernel at its own grid size; "
                 "configs 2/3 at <= 10M keys. traffic = the bytes the L2s read from the fabric, from the 32/64/128-B "
                 "read request counts (TCC_EA0_RDREQ_*B_sum; Infinity-Cache hits included), + WRITE_SIZE; "
                 "traffic_fetch_calibrated = FETCH_SIZE x the factor that turns the FETCH_SIZE of a same-run "
                 "ceiling pattern of known bytes into those bytes (fetch_factor, fetch_factor_from) + WRITE_SIZE. valu_busy = 4 x SQ_ACTIVE_INST_VALU / (%d SIMDs x GRBM_GUI_ACTIVE / %d XCDs) "
                 "(rocprof's VALUBusy formula); valu_busy_range = it divided by the same formula's reading on the "
                 "two VALU-saturating launches (half- and full-rate instructions): the kernel's true VALU "
                 "occupancy lies between. wait_frac = SQ_WAIT_ANY / SQ_WAVE_CYCLES" % (SIMDS, XCDS))


def valu_formula(c):
    if c.get("SQ_ACTIVE_INST_VALU") and c.get("GRBM_GUI_ACTIVE"):
        return 4.0 * c["SQ_ACTIVE_INST_VALU"] / (SIMDS * c["GRBM_GUI_ACTIVE"] / XCDS)
    return None


def pmc_calibration(pmc):
    """Factors from the ceiling patterns of known bytes: FETCH_SIZE (KiB) ->
    bytes read, WRITE_SIZE -> bytes written; the VALUBusy formula's reading on
    the saturating launches."""
    cal = {}
    for w, per_lane in CEIL_READ_PER_LANE.items():
        c = (pmc or {}).get(w)
        if c and c.get("FETCH_SIZE"):
            cal[w] = {"fetch_factor": round(c["_lanes"] * per_lane / (c["FETCH_SIZE"] * 1024.0), 4)}
            if c.get("WRITE_SIZE"):
                cal[w]["write_factor"] = round(c["_lanes"] * 16 / (c["WRITE_SIZE"] * 1024.0), 4)
    for w in ("ceil_valu_add", "ceil_valu_mul"):
        c = (pmc or {}).get(w)
        if c and valu_formula(c):
            cal[w] = {"valu_formula_reading": round(valu_formula(c), 4)}
    return cal


def read_bytes_by_size(c):
    """Bytes the L2s requested from the fabric, from the per-size request counts
    (32-, 64- and 128-B requests): exact for any access pattern, unlike
    FETCH_SIZE (which tallies a 128-B request as 64 B). None without them."""
    if all(c.get(k) is not None for k in RDREQ[:3]):
        return 32.0 * c[RDREQ[0]] + 64.0 * c[RDREQ[1]] + 128.0 * c[RDREQ[2]]
    return None


def pmc_fields(c, algorithmic_bytes, fetch_factor=2.0, valu_sat=None):
    """Derived counters of one workload (c: per-launch medians, KiB for the sizes).
    traffic = the per-size read bytes + WRITE_SIZE when the request-size pass ran,
    else FETCH_SIZE x the calibrated factor + WRITE_SIZE."""
    out = {}
    rb = read_bytes_by_size(c)
    if c.get("WRITE_SIZE") is not None and (rb is not None or c.get("FETCH_SIZE") is not None):
        if c.get("FETCH_SIZE") is not None:
            out["traffic_fetch_calibrated"] = (fetch_factor * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0
        t = rb + c["WRITE_SIZE"] * 1024.0 if rb is not None else out["traffic_fetch_calibrated"]
        out["traffic"] = t
        out["traffic_from"] = "per-size read requests + WRITE_SIZE" if rb is not None else \
            "FETCH_SIZE x fetch_factor + WRITE_SIZE"
        if rb is not None:
            out["read_bytes"] = rb
            out["read_requests_32_64_128B"] = [c.get(k) for k in RDREQ[:3]]
        out["traffic_over_algorithmic"] = round(t / algorithmic_bytes, 4) if algorithmic_bytes else None
    v = valu_formula(c)
    if v is not None:
        out["valu_busy"] = round(v, 4)
        if valu_sat:
            out["valu_busy_range"] = [round(v / max(valu_sat), 4), round(v / min(valu_sat), 4)]
    if c.get("SQ_WAIT_ANY") and c.get("SQ_WAVE_CYCLES"):
        out["wait_frac"] = round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 4)
    return out


def limiter(frac_of_ceiling, valu_hi):
    """Which resource is closer to its ceiling: the HBM (the line's rate over
    the measured ceiling of its shape) or the VALU (upper estimate)."""
    if frac_of_ceiling is None:
        return "unknown (ceiling not measured in this run)"
    if valu_hi is None:
        return "hbm (valu not measured)"
    return "hbm" if frac_of_ceiling >= valu_hi else "valu"


# ---------------------------------------------------------------------------
def summarize(w, walls, devs, steps, keys_total):
    vals = [keys_total / t for t in walls]
    i_med = int(np.argsort(vals)[len(vals) // 2])
    per_launch = devs[i_med]
    ops = getattr(w, "ops_per_key", 1)
    return {
        "value": vals[i_med] * ops,
        "value_min": min(vals) * ops, "value_max": max(vals) * ops, "repeats": len(vals),
        "ms_per_step": 1e3 * walls[i_med] / steps,
        "kernel_us": per_launch * 1e6,
        "achieved_gbs": w.n * w.bytes_per_key / per_launch / 1e9,
        "bytes_per_key": w.bytes_per_key,
        "lanes": w.n,
        "kernel": w.kernel,
        "desc": w.desc,
        "enqueue_us_per_step": 1e6 * w.enqueue_s / steps,
        "unique_gbs": (w.unique_bytes / per_launch / 1e9) if getattr(w, "unique_bytes", None) else None,
    }


def roofline_of(name, r, results, pmc, cal, args):
    """roofline object of one line: algorithmic GB/s over the spec peak and
    over the ceiling of the same shape measured in this run; PMC traffic with
    a calibrated FETCH_SIZE factor; VALU busy (formula and calibrated range)."""
    cands = [c for c in CEILING_OF.get(name, []) if c in results]
    ceil_name = max(cands, key=lambda c: results[c]["achieved_gbs"]) if cands else None
    ceil = results.get(ceil_name) if ceil_name else None
    ro = {"bound": "hbm", "achieved": round(r["achieved_gbs"], 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
          "frac": round(r["achieved_gbs"] / HBM_PEAK_GBS, 4), "traffic": None,
          "bytes_per_key": round(r["bytes_per_key"], 2), "kernel": r["kernel"],
          "kernel_us": round(r["kernel_us"], 2),
          "kernel_us_note": "HIP events on the launch stream around the K back-to-back launches / K (inter-kernel "
                            "gaps included)"}
    if name.startswith("ceil_valu"):
        ro["bound"], ro["unit"], ro["peak"] = "valu", "lane-ops/s", None
        ro["achieved"], ro["frac"] = r["value"], None
    if r.get("unique_gbs"):
        # each distinct row counted once (keys + distinct rows + records): what HBM must deliver at least.
        # This is the line's headline fraction: the per-key bytes count a row ~5 keys share
        # once per key, and those repeats come from the caches, not HBM (frac_per_key keeps that reading).
        ro["unique_gbs"] = round(r["unique_gbs"], 1)
        ro["frac_unique"] = round(r["unique_gbs"] / HBM_PEAK_GBS, 4)
        ro["frac_per_key"] = ro["frac"]
        ro["frac"] = ro["frac_unique"]
    if ceil is not None:
        ro["copy_ceiling"] = {"workload": ceil_name, "gbs": round(ceil["achieved_gbs"], 1),
                              "kernel_us": round(ceil["kernel_us"], 2)}
        ro["frac_of_copy_ceiling"] = round(r["achieved_gbs"] / ceil["achieved_gbs"], 4)
        if r.get("unique_gbs") and ceil.get("unique_gbs"):
            ro["frac_of_ceiling_unique"] = round(r["unique_gbs"] / ceil["unique_gbs"], 4)
    elif name in CEILING_OF:
        ro["frac_of_copy_ceiling"] = None
        ro["copy_ceiling"] = "%s not measured in this run" % " / ".join(CEILING_OF[name])
    key = {"fixed16_hot": "fixed16", "shard1b": "fixed16", "ceil_copy_hot": "ceil_copy",
           "ceil_copy_1b": "ceil_copy", "ceil_copynt_hot": "ceil_copynt", "ceil_copynt_1b": "ceil_copynt"}.get(name, name)
    c = (pmc or {}).get(key)
    valu_sat = [cal[w]["valu_formula_reading"] for w in ("ceil_valu_add", "ceil_valu_mul") if w in cal]
    if c and len(c) > 1:
        lanes = c["_lanes"]
        fsrc = FETCH_CAL_OF.get(key, key if key in CEIL_READ_PER_LANE else None)
        ff = cal.get(fsrc, {}).get("fetch_factor") if fsrc else None
        f = pmc_fields(c, lanes * r["bytes_per_key"], ff if ff else 2.0, valu_sat if len(valu_sat) == 2 else None)
        ro["fetch_factor"] = ff if ff else 2.0
        ro["fetch_factor_from"] = fsrc if ff else "MI355X_MICROARCH.md (x2, 16-B streams; no calibration this run)"
        ro["fetch_size_raw"] = c.get("FETCH_SIZE", 0) * 1024.0
        ro["write_size"] = c.get("WRITE_SIZE", 0) * 1024.0
        if lanes == r["lanes"]:
            ro["traffic"] = f.get("traffic")
        else:
            ro["traffic_at_pmc_size"] = f.get("traffic")
            ro["pmc_lanes"] = lanes
        for k in ("traffic_over_algorithmic", "traffic_from", "traffic_fetch_calibrated", "read_bytes",
                  "read_requests_32_64_128B", "valu_busy", "valu_busy_range", "wait_frac"):
            if k in f:
                ro[k] = f[k]
    vr = ro.get("valu_busy_range")
    if name.startswith("ceil_"):
        ro["limiter"] = "n/a (a ceiling line: what its access shape moves)"
    else:
        ro["limiter"] = limiter(ro.get("frac_of_copy_ceiling"), vr[1] if vr else ro.get("valu_busy"))
    return ro


def build_line(args, world, n_gpus, shared, results, verified, per_rank, units, pmc, pmc_note, cpu, host_inc,
               shards):
    """rank 0's JSON line from the reduced results (pure: no GPU, tested on the CPU)."""
    head_name = "fixed16" if "fixed16" in results else next(iter(results))
    head = results[head_name]
    cal = pmc_calibration(pmc)
    roof = roofline_of(head_name, head, results, pmc, cal, args)
    roof["algorithmic_bytes_per_launch"] = int(head["bytes_per_key"] * args.keys16) if head_name == "fixed16" \
        else None
    roof["traffic_note"] = pmc_note
    secondary = {}
    for name, r in results.items():
        if name == head_name:
            continue
        secondary[name] = {"value": r["value"], "value_min": r["value_min"], "value_max": r["value_max"],
                           "unit": units.get(name, "keys/s"), "ms_per_step": round(r["ms_per_step"], 4),
                           "desc": r["desc"], "roofline": roofline_of(name, r, results, pmc, cal, args),
                           "verified": verified.get(name)}
        if name == "shard1b":
            secondary[name]["scaling"] = "strong"
            secondary[name]["shards"] = shards
    all_ok = all(v["ok"] is True for v in verified.values()) if verified else None
    line = {
        "metric": METRIC,
        "value": head["value"],
        "unit": "keys/s",
        "n_gpus": n_gpus,
        "ranks": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "repeats": args.repeats,
        "value_min": head["value_min"],
        "value_max": head["value_max"],
        "ms_per_step": head["ms_per_step"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic: random key bytes generated on device (torch Philox), resident in HBM before timing",
        "config": {"workload": "BASELINE configs[1]: %d fixed 16-B keys per GPU per step, MurmurHash3_x64_128 "
                               "seed 12345 -> 16-B SHF_HASH (shf_make_hash batch), rotating over %d distinct "
                               "batches" % (args.keys16, max(1, args.rotate)),
                   "keys_per_gpu": args.keys16, "key_len": 16,
                   "parallelism": "dp%d (independent key shards, no collective)" % n_gpus},
        "roofline": roof,
        "verified": all_ok,
        "verification": verified,
        "cpu_baseline": cpu,
        "host_inclusive": host_inc,
        "secondary": secondary,
    }
    if cal:
        line["pmc_calibration"] = cal
    if world > 1:
        line["per_rank"] = per_rank
        spread = {}
        for name in results:
            ks = [pr["kernel_us"].get(name) for pr in per_rank if pr["kernel_us"].get(name)]
            if len(ks) == len(per_rank):
                spread[name] = round(max(ks) / min(ks), 4)
        line["slowest_over_fastest_rank"] = spread
        line["barrier_backend"] = args.dist_backend
    if shared:
        line["rehearsal"] = True
        line["rehearsal_note"] = "%d ranks shared %d GPU(s) (--allow-shared-gpu): throughput is not a " \
                                 "multi-GPU measurement" % (world, n_gpus)
    return line


LINE_MAX_BYTES = 4096  # the driver parses rank 0's stdout line from a ~10.7 KB stdout+stderr tail


def _sig(x, d=4):
    """x rounded to d significant digits (None and non-numbers pass through)."""
    if not isinstance(x, (int, float)) or isinstance(x, bool) or x == 0:
        return x
    return float("%.*g" % (d, x))


def compact_line(full, detail_path):
    """The stdout line (<= LINE_MAX_BYTES): the contract's fields, a compact
    roofline, cpu_baseline, host_inclusive and one short record per secondary
    line. Everything else (PMC counters, calibration, descriptions, per-rank
    records) stays in the detail file named by `detail`."""
    ro = full["roofline"]
    keep_ro = ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel", "kernel_us",
               "frac_of_copy_ceiling", "traffic_over_algorithmic", "valu_busy_range", "wait_frac", "limiter")
    roof = {k: _sig(ro.get(k), 5) for k in keep_ro if k in ro}
    if isinstance(ro.get("copy_ceiling"), dict):
        roof["copy_ceiling_gbs"] = ro["copy_ceiling"]["gbs"]
    if ro.get("algorithmic_bytes_per_launch"):
        roof["algorithmic_bytes_per_launch"] = ro["algorithmic_bytes_per_launch"]
    line = {k: full[k] for k in ("metric", "value", "unit", "n_gpus", "ranks", "steps", "warmup", "repeats",
                                 "ms_per_step", "higher_is_better", "scaling", "vs_baseline", "dtype") if k in full}
    line["value"] = _sig(line["value"], 6)
    line["ms_per_step"] = _sig(line["ms_per_step"], 5)
    line["value_min"], line["value_max"] = _sig(full["value_min"], 5), _sig(full["value_max"], 5)
    line["data"] = "synthetic (device Philox key bytes, resident in HBM before timing)"
    cfg = full["config"]
    line["config"] = {"workload": "BASELINE configs[1]: %d x 16-B keys/GPU/step, MurmurHash3_x64_128 seed 12345 -> "
                                  "SHF_HASH" % cfg["keys_per_gpu"],
                      "keys_per_gpu": cfg["keys_per_gpu"], "key_len": cfg["key_len"],
                      "parallelism": cfg["parallelism"]}
    line["roofline"] = roof
    line["verified"] = full.get("verified")
    cpu = full.get("cpu_baseline")
    if cpu:
        c = {"value": _sig(cpu["value"], 5), "unit": cpu["unit"], "cores": cpu["cores"], "kind": cpu["kind"],
             "sample": cpu["sample"][:120]}
        mt = next((v for k, v in cpu.items() if k.startswith("threads")), None)
        if mt:
            c["multi"] = {"value": _sig(mt["value"], 5), "cores": mt["cores"]}
        line["cpu_baseline"] = c
    else:
        line["cpu_baseline"] = None
    hi = full.get("host_inclusive")
    if hi:  # per line [G keys/s, frac_of_pcie]; the PCIe ceilings (GB/s) of the same run
        line["host_inclusive"] = {"unit": "G keys/s"}
        line["host_inclusive"].update({k: [round(v["value"] / 1e9, 3), v.get("frac_of_pcie")] for k, v in hi.items()
                                       if isinstance(v, dict) and "value" in v})
        if isinstance(hi.get("ceilings_gbs"), dict):
            c = hi["ceilings_gbs"]
            line["host_inclusive"]["pcie_gbs"] = {k: c[k] for k in ("h2d", "d2h", "both", "h2d_pageable", "zc_h2d",
                                                                    "zc_d2h", "zc_both") if k in c}
        line["host_inclusive"]["verified"] = hi.get("verified")
    sec, ceil = {}, {}
    for name, s in (full.get("secondary") or {}).items():
        r = s["roofline"]
        if name.startswith("ceil_"):
            ceil[name] = r["achieved"] if r.get("unit") == "GB/s" else _sig(s["value"], 4)
            continue
        e = {"value": _sig(s["value"], 5), "kernel_us": _sig(r.get("kernel_us"), 5),
             "frac": r.get("frac"), "frac_of_ceiling": r.get("frac_of_copy_ceiling")}
        if s["unit"] != full["unit"]:  # a secondary line's unit only where it is not the line's own (keys/s)
            e["unit"] = s["unit"]
        if r.get("traffic_over_algorithmic") is not None:
            e["traffic_x"] = r["traffic_over_algorithmic"]
        for k in ("frac_per_key", "frac_of_ceiling_unique"):
            if k in r:
                e[k] = r[k]
        e["verified"] = (s.get("verified") or {}).get("ok")
        if "scaling" in s:
            e["scaling"] = s["scaling"]
        if s.get("shards"):
            e["shards"] = s["shards"]
        if name == "hashwin16" and ro.get("kernel_us"):
            e["x_fixed16"] = round(r["kernel_us"] / ro["kernel_us"], 3)  # hash + order over the hash alone
        sec[name] = e
    line["secondary"] = sec
    line["ceilings_gbs"] = ceil
    if "slowest_over_fastest_rank" in full:
        sp = full["slowest_over_fastest_rank"]
        line["slowest_over_fastest_rank"] = {k: sp[k] for k in sp if not k.startswith("ceil_")}
        line["barrier_backend"] = full.get("barrier_backend")
    if full.get("rehearsal"):
        line["rehearsal"] = True
    line["detail"] = detail_path
    # hard cap: drop the least important blocks until the line fits
    for drop in ("ceilings_gbs", "slowest_over_fastest_rank", "host_inclusive"):
        if len(json.dumps(line)) <= LINE_MAX_BYTES:
            break
        line.pop(drop, None)
    while len(json.dumps(line)) > LINE_MAX_BYTES and line["secondary"]:
        line["secondary"].popitem()
    return line


def detail_path_for(args, world):
    return args.detail_out or os.path.join("gpurun_out", "bench_detail_n%d.json" % world)


def write_detail(path, full):
    """The full record (PMC counters, calibration, per-rank records) beside the line; best effort."""
    try:
        p = path if os.path.isabs(path) else os.path.join(ROOT, path)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "w") as f:
            json.dump(full, f, indent=1)
        return True
    except OSError:
        return False


def run_rank(args):
    rank, world, local, local_world = dist_env()
    import torch

    import sharedhashfile_amd as hb

    dev_idx, shared = plan_device(local, local_world, torch.cuda.device_count(), args.allow_shared_gpu)
    torch.cuda.set_device(dev_idx)
    dev = torch.device("cuda", dev_idx)
    dist, dist_dev = None, "cpu"
    if world > 1:
        import torch.distributed as tdist

        if args.dist_backend == "nccl":  # RCCL: barriers + max-reduces only, no data path
            if shared:
                raise SystemExit("bench.py: RCCL cannot run two ranks on one GPU; use --dist-backend gloo")
            tdist.init_process_group("nccl", device_id=dev)
            dist_dev = dev
        else:  # gloo on CPU tensors: no data crosses GPUs, so no RCCL init is needed
            tdist.init_process_group("gloo")
        dist = tdist
    hb.check_device()
    n_gpus = min(world, torch.cuda.device_count()) if shared else world

    wl = make_workloads(args, dev, rank, world)
    results, verified, mine = {}, {}, {"kernel_us": {}, "verified": {}}
    for w in wl:
        walls, devs, devs_local = time_workload(w, args.steps, args.warmup, args.repeats, dist, dist_dev,
                                                args.warmup_min_s)
        keys_total = (w.job_keys or w.n * world) * args.steps
        r = results[w.name] = summarize(w, walls, devs, args.steps, keys_total)
        mine["kernel_us"][w.name] = round(float(np.median(devs_local)) * 1e6, 2)
        log(args, "[bench] %s %.4g %s %.1fus %.0fGB/s" % (w.name, r["value"], getattr(w, "unit", "keys/s"),
                                                        r["kernel_us"], r["achieved_gbs"]))
        if not args.no_verify and w.verify is not None:
            try:
                ok, checked = w.verify()
            except Exception as e:  # noqa: BLE001
                ok, checked = None, 0
                log(args, "[bench] %s: verify unavailable: %s" % (w.name, e))
            mine["verified"][w.name] = ok
            if dist:
                t = torch.tensor([1 if ok else (0 if ok is False else -1)], dtype=torch.int64, device=dist_dev)
                dist.all_reduce(t, op=dist.ReduceOp.MIN)
                ok = True if int(t[0]) == 1 else (False if int(t[0]) == 0 else None)
            verified[w.name] = {"ok": ok, "samples_per_rank": checked}
            if ok is False:
                raise SystemExit("bench.py: %s outputs differ from the oracle" % w.name)
    shards = None
    sw = next((w for w in wl if w.name == "shard1b"), None)
    if sw is not None:
        shards = [list(sw.shard)]
    per_rank = None
    if dist:
        mine.update(rank=rank, device=dev_idx, device_name=torch.cuda.get_device_name(dev),
                    shard=list(sw.shard) if sw is not None else None)
        gathered = [None] * world
        dist.all_gather_object(gathered, mine)
        per_rank = sorted(gathered, key=lambda x: x["rank"])
        if sw is not None:
            shards = [pr["shard"] for pr in per_rank]

    if rank == 0:
        pmc, pmc_note = None, "not collected"
        if world == 1 and args.traffic == "auto":
            pmc, pmc_note = collect_pmc(args, list(results))
        cpu = cpu_baseline(args) if world == 1 and not args.no_cpu else None
        host_inc = time_host_inclusive(args, dev) if world == 1 and not args.no_host_inclusive else None
        units = {w.name: getattr(w, "unit", "keys/s") for w in wl}
        full = build_line(args, world, n_gpus, shared, results, verified, per_rank, units, pmc, pmc_note, cpu,
                          host_inc, shards)
        dpath = detail_path_for(args, world)
        if not write_detail(dpath, full):
            dpath = None
        line = compact_line(full, dpath)
        os.write(args.json_fd, (json.dumps(line) + "\n").encode())
    if dist:
        dist.barrier()
        dist.destroy_process_group()


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        n = args.gpus or 1
        if n > 1:  # spawn the ranks before anything touches the GPU
            return launch_ranks(argv, n)
    elif args.gpus is not None and args.gpus != int(env_world):
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%s" % (args.gpus, env_world))
    # stdout carries exactly one JSON line (rank 0's): whatever else writes to
    # fd 1 in a rank process (gloo's connection notices, library chatter) goes
    # to stderr
    sys.stdout.flush()
    args.json_fd = os.dup(1)
    os.dup2(2, 1)
    run_rank(args)
    return 0


if __name__ == "__main__":
    sys.exit(main())
