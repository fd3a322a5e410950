#!/bin/bash
set -o pipefail
OUT=gpurun_out/r3b_crb6
mkdir -p $OUT
export TMPDIR=/tmp
W=/tmp/wh_e2e_$$
echo "nproc $(nproc) affinity $(python3 -c 'import os; print(len(os.sched_getaffinity(0)))')"
run() {  # tag, env, args...
  local tag=$1; local e=$2; shift 2
  timeout -k 10 500 env $e python benchmarks/bench_e2e.py --rows 20000000 --files 4 --dir $W/$tag "$@" > $OUT/$tag.json 2> $OUT/$tag.err || { tail -20 $OUT/$tag.err; exit 1; }
  echo "$tag [$e]: $(tail -1 $OUT/$tag.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,2), "M ex/s, train_sec", round(d["train_sec"],3))')"
  grep "minibatches" $OUT/$tag.err | head -1
  rm -rf $W/$tag
}
run crb_t16 "WH_X=0" --format crb --minibatch 100000
run crb_t4 "WH_PARSE_THREADS=4" --format crb --minibatch 100000
run crb_t8 "WH_PARSE_THREADS=8" --format crb --minibatch 100000
run crb_p2 "WH_PREFETCH_PARTS=2" --format crb --minibatch 100000
echo done
