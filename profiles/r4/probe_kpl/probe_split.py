#!/usr/bin/env python3
"""f3 in the HBM regime: the fused hash + row pre-probe (k_fixed16<kOutProbe>) against the
split form -- the hash (k_fixed16) then the probe of the stored hashes (k_probe_hashes) --
on bench.py's probe16_hbm index (128 tabs per window, 2 GiB of rows). HIP events on the
current stream, median of 20 launches after 3 warm-ups; outputs compared."""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import sharedhashfile_amd as hb  # noqa: E402
from sharedhashfile_amd.keygen import device_random_bytes  # noqa: E402
from sharedhashfile_amd.rowindex import synthetic_index  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return float(np.median(ts))


def main():
    dev = torch.device("cuda:0")
    res = {}
    for tabs, n in ((16, 10_000_128), (128, 10_000_128 - 256)):
        keys = device_random_bytes(n * 16, 31, dev)
        h = hb.hash_fixed(keys, 16)
        tab_slot, rows, n_slots, _ = synthetic_index(h, tabs_per_win=tabs)
        index = hb.RowIndex(n_slots, tab_slot, rows)
        out1 = torch.empty((n, 4), dtype=torch.int32, device=dev)
        out2 = torch.empty((n, 4), dtype=torch.int32, device=dev)
        hh = torch.empty((n, 2), dtype=torch.int64, device=dev)
        fused = timed(lambda: hb.probe_fixed(index, keys, 16, out=out1))
        hash_only = timed(lambda: hb.hash_fixed(keys, 16, out=hh))
        probe_only = timed(lambda: hb.probe_hashes(index, hh, out=out2))
        split = timed(lambda: (hb.hash_fixed(keys, 16, out=hh), hb.probe_hashes(index, hh, out=out2)))
        torch.cuda.synchronize()
        same = bool(torch.equal(out1, out2))
        res["tabs%d" % tabs] = {"n": n, "fused_us": fused, "hash_us": hash_only, "probe_hashes_us": probe_only,
                                "split_us": split, "same": same}
        print("tabs %d: fused %.1f us, split %.1f us (hash %.1f + probe of hashes %.1f), same %s"
              % (tabs, fused, split, hash_only, probe_only, same), flush=True)
        del index, rows, tab_slot, keys, h
        torch.cuda.empty_cache()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
