#!/bin/bash
set -o pipefail
OUT=gpurun_out/r3b_crb2
mkdir -p $OUT
export TMPDIR=/tmp
W=/tmp/wh_e2e_$$
run() {  # tag, env, args...
  local tag=$1; local e=$2; shift 2
  timeout -k 10 300 env WH_INGEST_TIMING=1 $e python benchmarks/bench_e2e.py --rows 4000000 --files 4 --dir $W/$tag "$@" > $OUT/$tag.json 2> $OUT/$tag.err || { tail -20 $OUT/$tag.err; exit 1; }
  echo "$tag [$e]: $(tail -1 $OUT/$tag.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,2), "M ex/s, train_sec", round(d["train_sec"],3))')"
  grep "minibatches" $OUT/$tag.err | head -1
  rm -rf $W/$tag
}
run crb_dif_old "WH_CRB_BLOCKITER=0" --format crb --model difacto --minibatch 100000
run crb_dif_new "WH_X=0" --format crb --model difacto --minibatch 100000
run txt_dif "WH_X=0" --model difacto --minibatch 100000
run crb_dif_noshuf "WH_X=0" --format crb --model difacto --minibatch 100000 --rand-shuffle 0
echo done
