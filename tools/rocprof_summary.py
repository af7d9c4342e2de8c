#!/usr/bin/env python3
"""Compact rocprofv3 --stats kernel summary (short names, avg/min/max in us).

    python tools/rocprof_summary.py <kernel_stats.csv> > summary.md
"""
import csv
import sys


def short(name):
    name = name.replace("void ", "")
    if name.startswith("shfhb::"):
        return name.split("(")[0].replace("shfhb::", "")
    return name.split("(")[0][:60]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    print("| kernel | calls | avg us | min us | max us | % time |")
    print("|---|---|---|---|---|---|")
    for r in rows:
        print("| `%s` | %s | %.1f | %.1f | %.1f | %.1f |" % (
            short(r["Name"]), r["Calls"], float(r["AverageNs"]) / 1e3, float(r["MinNs"]) / 1e3,
            float(r["MaxNs"]) / 1e3, float(r["Percentage"])))


if __name__ == "__main__":
    main()
