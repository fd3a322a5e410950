#!/bin/bash
# One box: linear multi-shard step (loopback 8, 10k rows) vs the heavy-id
# partition total (WH_LOC_HEAVY 128 default / 64 / 32 / 8).
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r6g; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10 300"
b() { $T python bench.py "$@" > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; return 1; }; tail -1 $OUT/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.2f M ex/s %.1f us/step' % (d['value']/1e6, 1000*d['ms_per_step']))"; }
for i in 1 2 3; do
  for h in 128 64 32 8; do
    r=$(WH_LOC_HEAVY=$h b --model linear --loopback 8) || exit 1; echo "lin_lb8 heavy=$h $r"
  done
done | tee $OUT/ab.txt || exit 1
echo all done
