#!/bin/bash
# e2e DiFacto / linear from Criteo files under ingest settings (A/B)
set -o pipefail
OUT=gpurun_out/${1:-r3b_e2e}
ROWS=${ROWS:-20000000}
mkdir -p $OUT
export TMPDIR=/tmp
W=/tmp/wh_e2e_$$
run() {  # tag, env, args...
  local tag=$1; local e=$2; shift 2
  timeout -k 10 400 env $e python benchmarks/bench_e2e.py --rows $ROWS --files 4 --dir $W/$tag "$@" > $OUT/$tag.json 2> $OUT/$tag.err || { tail -20 $OUT/$tag.err; exit 1; }
  echo "$tag [$e]: $(tail -1 $OUT/$tag.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,2), "M ex/s, train_sec", round(d["train_sec"],3))')"
  grep "minibatches" $OUT/$tag.err | head -1
  rm -rf $W/$tag
}
run dif_base "WH_X=0" --model difacto --minibatch 100000
run dif_depth6 "WH_TEXT_DEPTH=6" --model difacto --minibatch 100000
run dif_noshuf "WH_X=0" --model difacto --minibatch 100000 --rand-shuffle 0
run lin10k_base "WH_X=0" --minibatch 10000
run lin10k_depth6 "WH_TEXT_DEPTH=6" --minibatch 10000
echo done
