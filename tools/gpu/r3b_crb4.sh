#!/bin/bash
set -o pipefail
OUT=gpurun_out/r3b_crb4
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 python tools/microbench/ingest_difacto_probe.py criteo 1000000 10 || exit $?
timeout -k 10 300 python tools/microbench/ingest_difacto_probe.py crb 1000000 10 || exit $?
timeout -k 10 300 python tools/microbench/ingest_difacto_probe.py crb 1000000 0 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 tools/microbench/ingest_difacto_probe.py crb 1000000 10 > $OUT/prof.log 2>&1 || exit $?
python3 - <<'PY'
import csv
for r in list(csv.DictReader(open('gpurun_out/r3b_crb4/prof/run_kernel_stats.csv')))[:15]:
    print("  %-58s %6s %9.1f %9.1f" % (r['Name'][:58], r['Calls'], float(r['AverageNs'])/1e3, float(r['TotalDurationNs'])/1e6))
PY
