#!/bin/bash
# linear at minibatch 10000: forward lanes per row / tile table A/B
set -o pipefail
OUT=gpurun_out/r3b_lin
mkdir -p $OUT
for i in 1 2; do
  for v in "A:WH_X=0" "B:WH_LIN_FWD_G=16" "C:WH_LIN_FWD_G=32" "D:WH_LD_TABLE=512" "E:WH_LIN_FWD_G=32 WH_LD_TABLE=512"; do
    n=${v%%:*}; e=${v#*:}
    timeout -k 10 300 env $e python bench.py --model linear > $OUT/$n.$i.log 2>&1 || exit $?
    echo "$n $i [$e] $(tail -1 $OUT/$n.$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,2), round(d["ms_per_step"]*1e3,1), "us")')"
  done
done
timeout -k 10 300 env WH_LIN_FWD_G=32 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --model linear > $OUT/prof.log 2>&1 || exit $?
python3 - <<'PY'
import csv
for r in list(csv.DictReader(open('gpurun_out/r3b_lin/prof/run_kernel_stats.csv')))[:8]:
    print("%-60s %6s %9.1f" % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))
PY
