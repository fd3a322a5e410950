#!/bin/bash
# Host API trace of the native vs Python multi-shard DiFacto step over the
# 1-rank RCCL loopback: which HIP calls block the host, and for how long.
set -o pipefail
OUT=gpurun_out/r4k; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10"
$T 300 rocprofv3 --hip-trace --kernel-trace --stats -d $OUT/nat -o run --output-format csv -- python bench.py --steps 60 --prewarm 200 --loopback 8 --loopback-rccl > $OUT/nat.log 2>&1 || exit $?
WH_PSX_NATIVE=0 $T 300 rocprofv3 --hip-trace --kernel-trace --stats -d $OUT/py -o run --output-format csv -- python bench.py --steps 60 --prewarm 200 --loopback 8 --loopback-rccl > $OUT/py.log 2>&1 || exit $?
tail -1 $OUT/nat.log; tail -1 $OUT/py.log
echo all done
