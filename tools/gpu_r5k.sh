#!/bin/bash
# One box: native DiFacto step with the AUC on its own stream vs the Python step,
# identity and RCCL loopbacks; P = 1 reference.
set -o pipefail
OUT=gpurun_out/r5k; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10 300"
b() { $T python bench.py "$@" 2>&1 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.2f M ex/s %.1f us/step' % (d['value']/1e6, 1000*d['ms_per_step']))"; }
for i in 1 2; do
  echo "lb8_nat $(b --loopback 8)" || exit 1
  echo "lb8_py $(WH_PSX_NATIVE=0 b --loopback 8)" || exit 1
  echo "rccl_nat $(WH_PSX_NATIVE=1 b --loopback 8 --loopback-rccl)" || exit 1
  echo "rccl_py $(b --loopback 8 --loopback-rccl)" || exit 1
  echo "p1 $(b)" || exit 1
done | tee $OUT/ab.txt || exit 1
echo all done
