#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats CSV run into a per-step table.

    python tools/prof_summary.py <prof_dir> <steps> [title]  > profiles/<name>.txt

Reads <prof_dir>/*kernel_trace.csv; prints calls, us/step, share, and (from the
trace) VGPR / LDS / grid size of each kernel plus the busy-time/step total.
"""
import csv
import glob
import sys
from collections import defaultdict


def main():
    d, steps = sys.argv[1], int(sys.argv[2])
    title = sys.argv[3] if len(sys.argv) > 3 else d
    tr = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)
    if not tr:
        sys.exit("no kernel_trace.csv under " + d)
    tot = defaultdict(int)
    calls = defaultdict(int)
    meta = {}
    t_first, t_last = None, None
    for row in csv.DictReader(open(tr[0])):
        n = row["Kernel_Name"]
        s, e = int(row["Start_Timestamp"]), int(row["End_Timestamp"])
        tot[n] += e - s
        calls[n] += 1
        meta[n] = (row.get("VGPR_Count"), row.get("Accum_VGPR_Count"), row.get("LDS_Block_Size"),
                   row.get("Grid_Size_X"), row.get("Workgroup_Size_X"))
        t_first = s if t_first is None else min(t_first, s)
        t_last = e if t_last is None else max(t_last, e)
    busy = sum(tot.values())
    print(title)
    print("kernel busy time per step: %.1f us (over %d profiled steps incl. warmup)" %
          (busy / 1e3 / steps, steps))
    print("%-78s %6s %10s %6s %5s %5s %6s %9s" % ("kernel", "calls", "us/step", "%", "vgpr",
                                                  "agpr", "lds", "grid"))
    for n, t in sorted(tot.items(), key=lambda kv: -kv[1]):
        v, a, l, g, w = meta[n]
        print("%-78s %6d %10.1f %5.1f%% %5s %5s %6s %9s" % (n[:78], calls[n], t / 1e3 / steps,
                                                           100.0 * t / busy, v, a, l, g))


if __name__ == "__main__":
    main()
