#!/bin/bash
# Round-4 measurements: same-box P=1 vs loopback-8 (DiFacto and linear at 10k),
# host profiles of the multi-shard step, kernel traces, PMC passes.
set -o pipefail
OUT=gpurun_out/r4b; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
b() { timeout -k 10 300 python bench.py "$@" 2>&1 | tail -1; }
echo "p1 $(b)" > $OUT/bench.txt || exit 1
echo "lb8 $(b --loopback 8)" >> $OUT/bench.txt || exit 1
echo "p1 $(b)" >> $OUT/bench.txt || exit 1
echo "lb8 $(b --loopback 8)" >> $OUT/bench.txt || exit 1
echo "lin_p1 $(b --model linear)" >> $OUT/bench.txt || exit 1
echo "lin_lb8 $(b --model linear --loopback 8)" >> $OUT/bench.txt || exit 1
echo "lin_p1 $(b --model linear)" >> $OUT/bench.txt || exit 1
echo "lin_lb8 $(b --model linear --loopback 8)" >> $OUT/bench.txt || exit 1
WH_HOST_PROFILE=$OUT/hp_lb8 timeout -k 10 300 python bench.py --loopback 8 > /dev/null 2>&1 || exit $?
WH_HOST_PROFILE=$OUT/hp_lin_lb8 timeout -k 10 300 python bench.py --model linear --loopback 8 > /dev/null 2>&1 || exit $?
WH_HOST_PROFILE=$OUT/hp_p1 timeout -k 10 300 python bench.py > /dev/null 2>&1 || exit $?
for cfg in "p1:" "lb8:--loopback 8" "lin_lb8:--model linear --loopback 8"; do
  t=${cfg%%:*}; a=${cfg#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$t -o run -- python3 bench.py --steps 100 $a > $OUT/kt_$t.log 2>&1 || exit $?
done
bash tools/gpu_pmc.sh r4b/pmc --steps 20 --warmup 2 --prewarm 300 || exit $?
echo all done
