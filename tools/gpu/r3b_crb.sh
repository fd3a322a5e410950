#!/bin/bash
set -o pipefail
OUT=gpurun_out/r3b_crb
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ingest.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
W=/tmp/wh_e2e_$$
run() {  # tag, env, args...
  local tag=$1; local e=$2; shift 2
  timeout -k 10 500 env WH_INGEST_TIMING=1 $e python benchmarks/bench_e2e.py --rows 20000000 --files 4 --dir $W/$tag "$@" > $OUT/$tag.json 2> $OUT/$tag.err || { tail -20 $OUT/$tag.err; exit 1; }
  echo "$tag [$e]: $(tail -1 $OUT/$tag.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,2), "M ex/s, train_sec", round(d["train_sec"],3))')"
  grep "minibatches" $OUT/$tag.err | head -1
  grep "ingest" $OUT/$tag.err | awk '{r+=$6; w+=$9; q+=$13} END {print "producers: read", r, "work", w, "full", q}'
  rm -rf $W/$tag
}
run crb "WH_X=0" --format crb --minibatch 100000
run crb_dif "WH_X=0" --format crb --model difacto --minibatch 100000
run lin100k "WH_X=0" --minibatch 100000
echo done
