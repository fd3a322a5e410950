#!/bin/bash
# End-to-end from files (bench_e2e.py): linear at the published minibatch
# (10k) and at 100k, DiFacto, and CRB input; each prints the JSON line and the
# worker's per-stage summary.
set -o pipefail
OUT=gpurun_out/${1:-r3e}
ROWS=${ROWS:-4000000}
mkdir -p $OUT
export TMPDIR=/tmp
W=/tmp/wh_e2e_$$
run() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 400 python benchmarks/bench_e2e.py --rows $ROWS --files 4 --dir $W/$tag "$@" > $OUT/$tag.json 2> $OUT/$tag.err || { tail -20 $OUT/$tag.err; exit 1; }
  echo "$tag: $(tail -1 $OUT/$tag.json | cut -c1-220)"
  grep "minibatches" $OUT/$tag.err | head -2
  rm -rf $W/$tag
}
run lin10k --minibatch 10000
run lin100k --minibatch 100000
run difacto --model difacto --minibatch 100000
run crb --format crb --minibatch 100000
echo done
