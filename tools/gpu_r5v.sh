#!/bin/bash
# One box: kernel timeline of the linear multi-shard step (loopback 8) and
# of the 1-shard linear step, for the GPU time per step.
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5v; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10 300"
$T rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/lb8 -o run -- python bench.py --model linear --loopback 8 --steps 200 > $OUT/lb8.log 2>&1 || { tail -5 $OUT/lb8.log; exit 1; }
$T rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/p1 -o run -- python bench.py --model linear --steps 200 > $OUT/p1.log 2>&1 || { tail -5 $OUT/p1.log; exit 1; }
python tools/step_timeline.py $OUT/lb8 k_synth_criteo 5 > $OUT/lb8_timeline.txt
python tools/step_timeline.py $OUT/p1 k_synth_criteo 5 > $OUT/p1_timeline.txt
tail -3 $OUT/lb8_timeline.txt; tail -3 $OUT/p1_timeline.txt
echo all done
