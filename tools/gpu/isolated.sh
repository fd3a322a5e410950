#!/bin/bash
# Isolated kernel times of a bench.py configuration: every launch serialised
# (AMD_SERIALIZE_KERNEL=3) under rocprofv3 --kernel-trace; the per-kernel
# mean is written to gpurun_out/TAG/isolated.txt.
# Usage: bash tools/gpu/isolated.sh TAG [bench.py args]
set -o pipefail
TAG=$1; shift
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
AMD_SERIALIZE_KERNEL=3 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/ser" -o run -- \
  python3 "${GRAFT_REPO_ROOT:-$OLDPWD}/bench.py" --steps 30 --warmup 5 --prewarm 300 "$@" > "$OUT/ser.log" 2>&1 || exit $?
python3 - "$OUT" <<'PY'
import csv, glob, sys
from collections import defaultdict
out = sys.argv[1]
agg = defaultdict(lambda: [0, 0.0])
for f in glob.glob(out + "/ser/**/*kernel_trace.csv", recursive=True):
    for x in csv.DictReader(open(f)):
        n = x["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:60]
        agg[n][0] += 1
        agg[n][1] += (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e3
# steps = the most common call count (a kernel launched twice per step, e.g.
# the copies, must not set it)
from collections import Counter
steps = Counter(c for c, _ in agg.values()).most_common(1)[0][0]
with open(out + "/isolated.txt", "w") as fo:
    tot = 0.0
    for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        if c < steps // 2:
            continue
        tot += t / steps
        fo.write("%-60s %5d %8.1f us/call %8.1f us/step\n" % (n, c, t / c, t / steps))
    fo.write("per-step kernel total %.1f us (%d steps)\n" % (tot, steps))
print(open(out + "/isolated.txt").read())
PY
