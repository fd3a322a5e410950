#!/bin/bash
set -o pipefail
OUT=gpurun_out/r3b_crb5
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_ingest.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
W=/tmp/wh_e2e_$$
run() {  # tag, env, args...
  local tag=$1; local e=$2; shift 2
  timeout -k 10 500 env $e python benchmarks/bench_e2e.py --rows 20000000 --files 4 --dir $W/$tag "$@" > $OUT/$tag.json 2> $OUT/$tag.err || { tail -20 $OUT/$tag.err; exit 1; }
  echo "$tag [$e]: $(tail -1 $OUT/$tag.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,2), "M ex/s, train_sec", round(d["train_sec"],3))')"
  grep "minibatches" $OUT/$tag.err | head -1
  rm -rf $W/$tag
}
run crb_dif "WH_X=0" --format crb --model difacto --minibatch 100000
run crb_lin "WH_X=0" --format crb --minibatch 100000
run crb_lin_old "WH_CRB_BLOCKITER=0" --format crb --minibatch 100000
run txt_dif "WH_X=0" --model difacto --minibatch 100000
echo done
