#!/bin/bash
# One box: where the native DiFacto step's host blocks (AUC side launches):
# AUC on the lent count stream (default) / its own stream / the compute stream.
set -o pipefail
OUT=gpurun_out/r5j; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10 300"
for v in "dflt|WH_X=0" "own|WH_PSX_AUC_OWN=1" "s|WH_PSX_AUC=s"; do
  IFS='|' read -r n e <<< "$v"
  env $e WH_STEP_TIMING=1 $T python bench.py --loopback 8 --steps 60 --warmup 20 --prewarm 200 > $OUT/$n.log 2>&1 || exit 1
  echo "$n: $(tail -1 $OUT/$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.2f M ex/s' % (d['value']/1e6))")"
  grep "host us" $OUT/$n.log | head -3
done
b() { $T python bench.py "$@" 2>&1 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.2f M ex/s %.1f us/step' % (d['value']/1e6, 1000*d['ms_per_step']))"; }
for i in 1 2; do
  echo "lb8_dflt $(b --loopback 8)"; echo "lb8_aucS $(WH_PSX_AUC=s b --loopback 8)"; echo "lb8_aucown $(WH_PSX_AUC_OWN=1 b --loopback 8)"
  echo "rccl_nat_aucS $(WH_PSX_NATIVE=1 WH_PSX_AUC=s b --loopback 8 --loopback-rccl)"; echo "rccl_py $(b --loopback 8 --loopback-rccl)"
  echo "p1 $(b)"
done | tee $OUT/ab.txt
echo all done
