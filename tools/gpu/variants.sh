#!/bin/bash
# Same-box A/B of environment variants of one bench, interleaved REPS times.
# Usage: bash tools/gpu/variants.sh TAG REPS "name:VAR=v VAR2=w" ... [-- bench.py args]
#   e.g. bash tools/gpu/variants.sh lin 2 "base:" "t2048:WH_LD_TABLE=2048" -- --model linear
set -o pipefail
TAG=$1; REPS=$2; shift 2
V=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do V+=("$1"); shift; done
[ "$1" = "--" ] && shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for i in $(seq 1 $REPS); do
  for v in "${V[@]}"; do
    n=${v%%:*}; e=${v#*:}
    timeout -k 10 300 env WH_VARIANT=$n $e python bench.py "$@" > $OUT/$n.$i.log 2>&1 || exit $?
    echo "$n $i [$e] $(tail -1 $OUT/$n.$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,2), "M", round(d["ms_per_step"]*1e3,1), "us/step")')"
  done
done
