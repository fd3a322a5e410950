#!/bin/bash
# Headline A/B of the training AUC's placement: device chain
# (WH_AUC_HOST_THREADS=0) vs host threads, benches interleaved.
set -o pipefail
OUT=gpurun_out/auc_ab
mkdir -p $OUT
timeout -k 10 60 ./tools/microbench/auc_host_bench > $OUT/micro.log 2>&1 || exit $?
cat $OUT/micro.log
nproc; cat /proc/cpuinfo | grep -m1 "model name"
for i in 1 2; do
  for v in "WH_AUC_HOST_THREADS=0" "WH_AUC_HOST_THREADS=2" "WH_AUC_HOST_THREADS=4"; do
    tag=$(echo $v | tr ' =' '__')
    timeout -k 10 300 env $v python bench.py "$@" > $OUT/$tag.$i.log 2>&1 || exit $?
    echo "$v | $i $(tail -1 $OUT/$tag.$i.log | cut -c1-110)"
  done
done
