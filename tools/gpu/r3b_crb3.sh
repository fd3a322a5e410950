#!/bin/bash
set -o pipefail
OUT=gpurun_out/r3b_crb3
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
W=/tmp/wh_e2e_$$
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 benchmarks/bench_e2e.py --rows 4000000 --files 4 --dir $W/x --format crb --model difacto --minibatch 100000 > $OUT/run.json 2> $OUT/run.err || { tail -20 $OUT/run.err; exit 1; }
grep minibatches $OUT/run.err | head -2
ls -R $OUT/prof | head
python3 - <<'PY'
import csv,glob
for f in glob.glob('gpurun_out/r3b_crb3/prof/**/*kernel_stats.csv', recursive=True):
    print(f)
    for r in list(csv.DictReader(open(f)))[:15]:
        print("  %-58s %6s %9.1f %9.1f" % (r['Name'][:58], r['Calls'], float(r['AverageNs'])/1e3, float(r['TotalDurationNs'])/1e6))
PY
