#!/bin/bash
set -o pipefail
OUT=gpurun_out/r3b_parse
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 120 python tools/microbench/parse_bench.py 100000 50 || exit $?
timeout -k 10 120 python tools/microbench/parse_bench.py 1000000 10 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 tools/microbench/parse_bench.py 100000 50 > $OUT/prof.log 2>&1 || exit $?
python3 - <<'PY'
import csv
for r in list(csv.DictReader(open('gpurun_out/r3b_parse/prof/run_kernel_stats.csv')))[:12]:
    print("%-60s %6s %9.1f" % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))
PY
