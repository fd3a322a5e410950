#!/bin/bash
# One box: linear at 10k rows, multi-shard step (loopback 8) vs P = 1,
# interleaved, for the same-box ratio.
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r6c; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10 300"
b() { $T python bench.py "$@" > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; return 1; }; tail -1 $OUT/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.2f M ex/s %.1f us/step' % (d['value']/1e6, 1000*d['ms_per_step']))"; }
for i in 1 2 3 4; do
  r=$(b --model linear --loopback 8) || exit 1; echo "lin_lb8 $r"
  r=$(b --model linear) || exit 1; echo "lin_p1 $r"
done | tee $OUT/ab.txt || exit 1
echo all done
