#!/usr/bin/env python3
"""Summarise rocprofv3 --stats kernel_stats.csv files: kernel, calls, mean us,
total ms (names shortened). Usage: python tools/kstats.py DIR [N]"""
import csv
import glob
import sys


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0][:58]


def main():
    d = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    for f in sorted(glob.glob(d + "/**/*kernel_stats.csv", recursive=True)):
        rows = list(csv.DictReader(open(f)))
        tot = sum(float(r["TotalDurationNs"]) for r in rows)
        print("# %s: %d kernels, %.2f ms total" % (f.split("/")[-3] if "/" in f else f, len(rows),
                                                   tot / 1e6))
        for r in rows[:top]:
            print("%-60s %7s %10.1f us %9.2f ms %5.1f%%" % (
                short(r["Name"]), r["Calls"], float(r["AverageNs"]) / 1e3,
                float(r["TotalDurationNs"]) / 1e6, float(r["Percentage"])))


if __name__ == "__main__":
    main()
