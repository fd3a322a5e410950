#!/bin/bash
# CRB / text e2e A/B over the SAME files (generated once per format)
set -o pipefail
OUT=gpurun_out/r3b_crb7
mkdir -p $OUT
export TMPDIR=/tmp
W=/tmp/wh_e2e_$$
run() {  # tag, dir, env, args...
  local tag=$1; local d=$2; local e=$3; shift 3
  timeout -k 10 500 env $e python benchmarks/bench_e2e.py --rows 20000000 --files 4 --dir $W/$d --reuse "$@" > $OUT/$tag.json 2> $OUT/$tag.err || { tail -20 $OUT/$tag.err; exit 1; }
  echo "$tag [$e]: $(tail -1 $OUT/$tag.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,2), "M ex/s, train_sec", round(d["train_sec"],3), "gen", round(d["datagen_sec"],1))')"
  grep "minibatches" $OUT/$tag.err | head -1
}
run crb_a1 crb "WH_X=0" --format crb --minibatch 100000
run crb_old1 crb "WH_CRB_BLOCKITER=0" --format crb --minibatch 100000
run crb_a2 crb "WH_X=0" --format crb --minibatch 100000
run crb_old2 crb "WH_CRB_BLOCKITER=0" --format crb --minibatch 100000
run crb_dif crb "WH_X=0" --format crb --model difacto --minibatch 100000
rm -rf $W/crb
run txt_dif1 txt "WH_X=0" --model difacto --minibatch 100000
run txt_dif2 txt "WH_X=0" --model difacto --minibatch 100000
run txt_dif_r1 txt "WH_TEXT_READERS=1" --model difacto --minibatch 100000
run txt_lin10k txt "WH_X=0" --minibatch 10000
rm -rf $W
echo done
