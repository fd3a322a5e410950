#!/bin/bash
# A/B of an environment setting on one box, benches interleaved.
# Usage: bash tools/gpu/env_ab.sh TAG "VAR=val ..." [bench args]
set -o pipefail
TAG=${1:-envab}; ENVB=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
for i in 1 2; do
  timeout -k 10 300 python bench.py "$@" > $OUT/a.$i.log 2>&1 || exit $?
  echo "A $i $(tail -1 $OUT/a.$i.log | cut -c1-150)"
  timeout -k 10 300 env $ENVB python bench.py "$@" > $OUT/b.$i.log 2>&1 || exit $?
  echo "B $i $(tail -1 $OUT/b.$i.log | cut -c1-150)"
done
