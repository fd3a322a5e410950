#!/usr/bin/env python3
"""Per-kernel sums of rocprofv3 --pmc counters (counter_collection.csv):
python tools/pmc_kernel.py DIR SUBSTRING -> counter totals for matching kernels
(summed over dispatches) and the dispatch count."""
import csv
import glob
import sys
from collections import defaultdict


def main():
    d, sub = sys.argv[1], sys.argv[2]
    tot = defaultdict(float)
    disp = set()
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if sub not in r["Kernel_Name"]:
                continue
            disp.add(r["Dispatch_Id"])
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
    print("# %s: %d dispatches matching %r" % (d, len(disp), sub))
    for k in sorted(tot):
        print("%-32s %16.0f" % (k, tot[k]))


if __name__ == "__main__":
    main()
