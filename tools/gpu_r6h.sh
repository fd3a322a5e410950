#!/bin/bash
# One box: the linear loopback-8 step's two run states (~165 vs ~190
# us/step): host split per run, to tell GPU from host lateness.
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r6h; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10 300"
for i in 1 2 3 4 5 6; do
  WH_STEP_TIMING=1 $T python bench.py --model linear --loopback 8 > $OUT/t$i.log 2>&1 || { tail -5 $OUT/t$i.log; exit 1; }
  v=$(tail -1 $OUT/t$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.2f M %.1f us/step' % (d['value']/1e6, 1000*d['ms_per_step']))")
  echo "run $i $v | $(grep 'host us' $OUT/t$i.log | tail -1)"
done | tee $OUT/ab.txt || exit 1
echo all done
