#!/bin/bash
# One box: linear multi-shard step (loopback 8, 10k rows) vs the localize
# partition count: WH_LOC_NNZ_PART / WH_LOC_PART_IDS sweep, plus a kernel
# timeline at 2048 non-zeros per partition.
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5w; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10 300"
b() { $T python bench.py "$@" > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; return 1; }; tail -1 $OUT/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.2f M ex/s %.1f us/step' % (d['value']/1e6, 1000*d['ms_per_step']))"; }
for i in 1 2; do
  for np in 16384 4096 2048 1024; do
    r=$(WH_LOC_NNZ_PART=$np b --model linear --loopback 8) || exit 1; echo "lin_lb8 nnz_part=$np $r"
  done
  r=$(WH_LOC_PART_IDS=512 b --model linear --loopback 8) || exit 1; echo "lin_lb8 part_ids=512 $r"
  r=$(WH_LOC_PART_IDS=512 WH_LOC_NNZ_PART=2048 b --model linear --loopback 8) || exit 1; echo "lin_lb8 part_ids=512 nnz_part=2048 $r"
done | tee $OUT/ab.txt || exit 1
WH_LOC_NNZ_PART=2048 $T rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/lb8 -o run -- python bench.py --model linear --loopback 8 --steps 200 > $OUT/lb8.log 2>&1 || { tail -5 $OUT/lb8.log; exit 1; }
python tools/step_timeline.py $OUT/lb8 k_synth_criteo 5 > $OUT/lb8_timeline.txt
cat $OUT/lb8_timeline.txt
echo all done
