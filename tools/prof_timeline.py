#!/usr/bin/env python3
"""Print the kernel timeline (start offset, duration, idle gap, queue) of one
step of a rocprofv3 trace: python tools/prof_timeline.py <db> [--step-kernel
k_fm_fwd] [--back 2]."""
import argparse
import sqlite3

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--step-kernel", default="k_fm_fwd")
ap.add_argument("--back", type=int, default=2)
a = ap.parse_args()
con = sqlite3.connect(a.db)
rows = con.execute("select name, start, end, queue_id from kernels order by start").fetchall()
marks = [r[1] for r in rows if a.step_kernel in r[0]]
t0, t1 = marks[-a.back - 1], marks[-a.back]
prev_end = None
for n, s, e, q in rows:
    if t0 <= s < t1:
        n = n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:48]
        gap = (s - prev_end) / 1e3 if prev_end else 0
        print("%8.1f %7.1f gap %6.1f  q%s %s" % ((s - t0) / 1e3, (e - s) / 1e3, gap, q, n))
        prev_end = max(prev_end or 0, e)
