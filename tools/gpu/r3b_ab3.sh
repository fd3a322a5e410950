#!/bin/bash
set -o pipefail
OUT=gpurun_out/r3b_ab3
mkdir -p $OUT
for i in 1 2; do
  for v in "A:" "B:GPU_MAX_HW_QUEUES=8" "C:WH_DIFACTO_BEGIN=late" "D:GPU_MAX_HW_QUEUES=8 WH_DIFACTO_BEGIN=late"; do
    n=${v%%:*}; e=${v#*:}
    timeout -k 10 300 env $e python bench.py > $OUT/$n.$i.log 2>&1 || exit $?
    echo "$n $i $e $(tail -1 $OUT/$n.$i.log | cut -c100-175)"
  done
done
