#!/bin/bash
# A/B on one box: the current tree vs the worktree in ab_old/ (built
# in-tree there), benches interleaved. Usage: bash tools/gpu_ab.sh TAG [bench args]
set -o pipefail
TAG=${1:-ab}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for i in 1 2; do
  for side in new old; do
    dir=.; [ $side = old ] && dir=ab_old
    (cd $dir && timeout -k 10 300 python bench.py "$@") > $OUT/$side.$i.log 2>&1 || exit $?
    echo "$side $i $(tail -1 $OUT/$side.$i.log | cut -c1-160)"
  done
done
