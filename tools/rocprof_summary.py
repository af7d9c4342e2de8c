#!/usr/bin/env python3
"""rocprofv3 kernel summary keyed by kernel AND launch grid.

    python tools/rocprof_summary.py <dir with *kernel_trace.csv> [--label L] > summary.md

rocprofv3 --stats names a kernel by its symbol only, so one row would lump a
10M-key k_fixed16 launch with a 1B-key one. Here every (kernel, Grid_Size_X)
pair is its own row, with the launch count and the average / min / max
duration from the kernel trace (End - Start), so a bench line's `kernel_us`
can be checked against the launches of exactly its shape.
"""
import argparse
import collections
import csv
import glob
import os


def short(name):
    name = name.replace("void ", "").replace("(anonymous namespace)::", "")
    if "shfhb::" in name:
        return name.split("(")[0].replace("shfhb::", "")
    return name.split("(")[0][:60]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("root")
    p.add_argument("--label", default="")
    a = p.parse_args()
    acc = collections.defaultdict(list)
    for f in glob.glob(os.path.join(a.root, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                dur = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3
                acc[(short(row["Kernel_Name"]), int(row.get("Grid_Size_X") or row.get("Grid_Size") or 0))].append(dur)
    total = sum(sum(v) for v in acc.values()) or 1.0
    if a.label:
        print("### %s\n" % a.label)
    print("| kernel | grid (work-items) | calls | avg us | min us | max us | % time |")
    print("|---|---|---|---|---|---|---|")
    for (k, g), v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
        print("| `%s` | %d | %d | %.1f | %.1f | %.1f | %.1f |" % (k, g, len(v), sum(v) / len(v), min(v), max(v),
                                                              100.0 * sum(v) / total))


if __name__ == "__main__":
    main()
