#!/usr/bin/env python3
"""Per-kernel PMC summary from rocprofv3 --pmc CSV passes (tools/gpu_pmc.sh).

    python tools/pmc_summary.py <pmc_dir> [top]   (pmc_dir holds p1..pN/)

Prints per kernel: time share, L2 hit rate, HBM read/write GB/s (FETCH_SIZE /
WRITE_SIZE are KiB; on gfx950 FETCH_SIZE can under-count wide streams up to
2x, so read bytes are a lower bound), float/int atomic requests and the wave
wait/busy split from the SQ counters.
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d):
    val = defaultdict(lambda: defaultdict(float))
    dur = defaultdict(float)
    for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
        seen = set()
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            val[k][r["Counter_Name"]] += float(r["Counter_Value"])
            did = (f, r["Dispatch_Id"])
            if did not in seen and f.endswith(("p1/run_counter_collection.csv",)):
                seen.add(did)
                dur[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    return val, dur


def main():
    d = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 15
    val, dur = load(d)
    tot = sum(dur.values()) or 1.0
    print("%-60s %7s %6s %7s %8s %8s %9s %6s %6s" % ("kernel", "us", "%", "L2hit", "rdGB/s",
                                                     "wrGB/s", "atomicReq", "wait%", "inst%"))
    for k, t in sorted(dur.items(), key=lambda kv: -kv[1])[:top]:
        c = val[k]
        hit, miss = c.get("TCC_HIT_sum", 0), c.get("TCC_MISS_sum", 0)
        hr = hit / (hit + miss) if hit + miss else 0
        rd = c.get("FETCH_SIZE", 0) * 1024 / (t * 1e-6) / 1e9 if t else 0
        wr = c.get("WRITE_SIZE", 0) * 1024 / (t * 1e-6) / 1e9 if t else 0
        wc = c.get("SQ_WAVE_CYCLES", 0)
        wait = 100 * c.get("SQ_WAIT_ANY", 0) / wc if wc else 0
        inst = 100 * c.get("SQ_ACTIVE_INST_ANY", 0) / wc if wc else 0
        print("%-60s %7.0f %5.1f%% %6.1f%% %8.0f %8.0f %9.0f %5.1f%% %5.1f%%" % (
            k[:60], t, 100 * t / tot, 100 * hr, rd, wr, c.get("TCC_EA0_ATOMIC_sum", 0), wait,
            inst))


if __name__ == "__main__":
    main()
