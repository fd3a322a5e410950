#!/bin/bash
# A/B on one box: hardware queues per process (HIP's default 4 vs 8) for the
# P=1 headline and the multi-shard steps (native / Python) over the loopbacks.
set -o pipefail
OUT=gpurun_out/r4l; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10"
b() { $T 300 python bench.py "$@" 2>&1 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.2f M ex/s %.1f us/step' % (d['value']/1e6, 1000*d['ms_per_step']))"; }
for i in 1 2; do
  for q in 4 8; do
    export GPU_MAX_HW_QUEUES=$q
    echo "q$q p1 $(b)" || exit 1
    echo "q$q rccl_native $(b --loopback 8 --loopback-rccl)" || exit 1
    echo "q$q rccl_python $(WH_PSX_NATIVE=0 b --loopback 8 --loopback-rccl)" || exit 1
    echo "q$q lb8_native $(b --loopback 8)" || exit 1
    echo "q$q lin_rccl_native $(b --loopback 8 --loopback-rccl --model linear)" || exit 1
    echo "q$q lin_lb8_native $(b --loopback 8 --model linear)" || exit 1
    echo "q$q lin_p1 $(b --model linear)" || exit 1
  done
done | tee $OUT/ab.txt || exit 1
echo all done
