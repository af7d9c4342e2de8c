#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSV output: median counter value per (kernel, grid).

    python tools/pmc_summary.py <dir containing *counter_collection.csv> [kernel-substring ...]
"""
import collections
import csv
import statistics
import glob
import os
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "").split("(")[0]
    return name.replace("void ", "").replace("shfhb::", "")


def main():
    root = sys.argv[1]
    want = sys.argv[2:]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                raw = row["Kernel_Name"]
                if want and not any(w in raw for w in want):
                    continue
                k = "%s  grid %s" % (short(raw), row.get("Grid_Size", "?"))
                acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, cs in sorted(acc.items()):
        print(k)
        for c, v in sorted(cs.items()):
            print("   %-28s %16.1f  (median of n=%d)" % (c, statistics.median(v), len(v)))


if __name__ == "__main__":
    main()
