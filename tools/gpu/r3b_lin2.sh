#!/bin/bash
set -o pipefail
OUT=gpurun_out/r3b_lin2
mkdir -p $OUT
for i in 1 2; do
  for v in "A:WH_X=0" "B:WH_LD_TABLE=2048" "C:WH_LINEAR_DIRECT_NNZ=0"; do
    n=${v%%:*}; e=${v#*:}
    timeout -k 10 300 env $e python bench.py --model linear > $OUT/$n.$i.log 2>&1 || exit $?
    echo "$n $i [$e] $(tail -1 $OUT/$n.$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,2), round(d["ms_per_step"]*1e3,1), "us")')"
  done
done
