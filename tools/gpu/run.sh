#!/bin/bash
# One GPU call, several bench.py configurations, each REPS times interleaved.
# Usage: bash tools/gpu/run.sh TAG REPS "name|ENV=v ...|bench args" ...
#   e.g. bash tools/gpu/run.sh base 2 "d1||" "lb8r||--loopback 8 --loopback-rccl" \
#          "lin8|WH_TIMING=step|--model linear --loopback 8"
# Logs go to gpurun_out/TAG/<name>.<i>.log; one summary line per run is
# printed and appended to gpurun_out/TAG/summary.txt. The first failing run
# ends the call (no retries).
set -o pipefail
TAG=$1; REPS=$2; shift 2
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/$TAG
mkdir -p "$OUT"
for i in $(seq 1 "$REPS"); do
  for spec in "$@"; do
    IFS='|' read -r n e a <<< "$spec"
    log=$OUT/$n.$i.log
    # shellcheck disable=SC2086
    timeout -k 10 300 env $e python bench.py $a > "$log" 2>&1 || { echo "FAIL $n $i"; tail -20 "$log"; exit 1; }
    s=$(tail -1 "$log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.2f M ex/s %.1f us/step" % (d["value"]/1e6, d["ms_per_step"]*1e3))')
    echo "$n $i [$e] [$a] $s" | tee -a "$OUT/summary.txt"
  done
done
