#!/bin/bash
# One box: native multi-shard DiFacto step, host phase timestamps (CLOCK_MONOTONIC)
# alongside a kernel trace, identity and RCCL loopbacks.
set -o pipefail
OUT=gpurun_out/r5i; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10 300"
WH_STEP_TIMING=2 $T rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$OUT/lb8 -o run -- python3 bench.py --loopback 8 --steps 60 --warmup 20 --prewarm 200 > $OUT/lb8.log 2>&1 || exit 1
WH_PSX_NATIVE=1 WH_STEP_TIMING=2 $T rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$OUT/rccl -o run -- python3 bench.py --loopback 8 --loopback-rccl --steps 60 --warmup 20 --prewarm 200 > $OUT/rccl.log 2>&1 || exit 1
grep -c "marks ns" $OUT/lb8.log $OUT/rccl.log
echo all done
