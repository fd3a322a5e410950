#!/bin/bash
# multi-rank rehearsal (gloo-staged, 2 and 4 ranks on one GPU) + loopback-8 benches
set -o pipefail
OUT=gpurun_out/r3b_multi
mkdir -p $OUT
bash tools/gpu_2rank.sh r3b_multi/two 2 4 || exit $?
for v in "lb8:--loopback 8" "lb8rccl:--loopback 8 --loopback-rccl" "lin_lb8:--loopback 8 --model linear --batch 100000"; do
  n=${v%%:*}; a=${v#*:}
  timeout -k 10 300 python bench.py $a > $OUT/$n.log 2>&1 || exit $?
  echo "$n $(tail -1 $OUT/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,2), d["ms_per_step"])')"
done
for q in 2 3; do
  timeout -k 10 300 env GPU_MAX_HW_QUEUES=$q python bench.py > $OUT/q$q.log 2>&1 || exit $?
  echo "hwq$q $(tail -1 $OUT/q$q.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,2), d["ms_per_step"])')"
done
