#!/bin/bash
# A/B on one box: native vs Python multi-shard step over the 1-rank RCCL
# loopback (blocking C0 exchange fix), localize XCD tile order on / off.
set -o pipefail
OUT=gpurun_out/r4f; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10"
b() { $T 300 python bench.py "$@" 2>&1 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.2f M ex/s %.1f us/step' % (d['value']/1e6, 1000*d['ms_per_step']))"; }
for i in 1 2 3; do
  echo "p1 $(b)"
  echo "p1_locxcd0 $(WH_LOC_XCD=0 b)"
  echo "rccl_native $(b --loopback 8 --loopback-rccl)"
  echo "rccl_python $(WH_PSX_NATIVE=0 b --loopback 8 --loopback-rccl)"
  echo "lin_rccl_native $(b --loopback 8 --loopback-rccl --model linear)"
  echo "lin_rccl_python $(WH_PSX_NATIVE=0 b --loopback 8 --loopback-rccl --model linear)"
done | tee $OUT/ab.txt
WH_STEP_TIMING=1 $T 300 python bench.py --loopback 8 --model linear > $OUT/lin_timing.log 2>&1 || exit $?
WH_STEP_TIMING=1 $T 300 python bench.py --loopback 8 > $OUT/dif_timing.log 2>&1 || exit $?
grep "host us" $OUT/lin_timing.log $OUT/dif_timing.log | tail -4
echo all done
