#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace (rocpd SQLite output) of a bench run.

    python tools/prof_summary.py <results.db> [--last-steps K --step-kernel NAME]

Reports, over the analysed window: per-kernel calls, total and mean time, and
the time per step (total / steps); the GPU busy fraction (union of kernel
intervals over the window's wall time) and the largest idle gaps. The window
is the whole trace, or the last K steps delimited by the K-th last dispatch of
--step-kernel (one launch per training step, e.g. the FM forward).
"""
import argparse
import sqlite3
import sys


def load(db):
    con = sqlite3.connect(db)
    cur = con.cursor()
    rows = cur.execute("select name, start, end, grid_x, workgroup_x, vgpr_count, "
                       "accum_vgpr_count, lds_size from kernels order by start").fetchall()
    return rows


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    n = n.split("(")[0]
    if len(n) > 70:
        n = n[:67] + "..."
    return n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last-steps", type=int, default=0)
    ap.add_argument("--step-kernel", default="k_fm_fwd")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    rows = load(a.db)
    if not rows:
        sys.exit("no kernels in the trace")
    steps = None
    if a.last_steps:
        marks = [r[1] for r in rows if a.step_kernel in r[0]]
        if len(marks) <= a.last_steps:
            sys.exit("only %d dispatches of %s" % (len(marks), a.step_kernel))
        t0, t1 = marks[-a.last_steps - 1], marks[-1]
        rows = [r for r in rows if t0 <= r[1] < t1]
        steps = a.last_steps
    t0 = min(r[1] for r in rows)
    t1 = max(r[2] for r in rows)
    agg = {}
    for name, s, e, gx, wx, vg, ag, lds in rows:
        k = short(name)
        d = agg.setdefault(k, [0, 0, gx // max(wx, 1), vg, ag, lds])
        d[0] += 1
        d[1] += e - s
    busy, cur_s, cur_e, gaps = 0, None, None, []
    for _, s, e, *_ in rows:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                gaps.append((s - cur_e, cur_e))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    wall = t1 - t0
    tot = sum(d[1] for d in agg.values())
    print("window: %.3f ms wall, %d dispatches, kernel sum %.3f ms, GPU busy %.1f%%%s" % (
        wall / 1e6, len(rows), tot / 1e6, 100.0 * busy / wall,
        "" if steps is None else ", %d steps -> %.1f us/step wall, %.1f us/step busy" % (
            steps, wall / 1e3 / steps, busy / 1e3 / steps)))
    print("%-70s %7s %10s %9s %9s %6s %4s %4s %6s" % ("kernel", "calls", "total_ms", "mean_us",
                                                     "us/step", "wgs", "vgpr", "agpr", "lds"))
    for k, d in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print("%-70s %7d %10.3f %9.2f %9s %6d %4d %4d %6d" % (
            k, d[0], d[1] / 1e6, d[1] / 1e3 / d[0],
            "%.1f" % (d[1] / 1e3 / steps) if steps else "-", d[2], d[3], d[4], d[5]))
    gaps.sort(reverse=True)
    print("largest idle gaps (us): " + ", ".join("%.1f" % (g / 1e3) for g, _ in gaps[:10]))
    if steps:
        print("idle per step: %.1f us in %d gaps" % ((wall - busy) / 1e3 / steps, len(gaps)))


if __name__ == "__main__":
    main()
