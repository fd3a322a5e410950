#!/bin/bash
# A/B on one box: native multi-shard step with C1..C3 on the issuing stream
# (default) vs on RCCL's internal stream (WH_PSX_A2A=async) vs the Python
# step, over the 1-rank RCCL loopback; then a kernel trace of the default.
set -o pipefail
OUT=gpurun_out/r4j; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10"
b() { $T 300 python bench.py "$@" 2>&1 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.2f M ex/s %.1f us/step' % (d['value']/1e6, 1000*d['ms_per_step']))"; }
for i in 1 2 3; do
  echo "rccl_native $(b --loopback 8 --loopback-rccl)" || exit 1
  echo "rccl_native_aucown $(WH_PSX_AUC_OWN=1 b --loopback 8 --loopback-rccl)" || exit 1
  echo "rccl_python $(WH_PSX_NATIVE=0 b --loopback 8 --loopback-rccl)" || exit 1
  echo "lb8_native $(b --loopback 8)" || exit 1
  echo "lb8_python $(WH_PSX_NATIVE=0 b --loopback 8)" || exit 1
  echo "lin_rccl_native $(b --loopback 8 --loopback-rccl --model linear)" || exit 1
  echo "lin_rccl_python $(WH_PSX_NATIVE=0 b --loopback 8 --loopback-rccl --model linear)" || exit 1
done | tee $OUT/ab.txt || exit 1
$T 300 rocprofv3 --kernel-trace -d $OUT/nat -o run --output-format csv -- python bench.py --steps 60 --prewarm 200 --loopback 8 --loopback-rccl > $OUT/nat.log 2>&1 || exit $?
echo all done
