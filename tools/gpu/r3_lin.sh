#!/bin/bash
# linear single-GPU step: sizes x step kinds, plus kernel traces of the direct step
set -o pipefail
OUT=gpurun_out/${1:-r3l}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_apps_gpu.py -m gpu -q -k "native_linear or leaf_walk or gbdt" --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -1 $OUT/tests.log
[ $rc -le 1 ] || exit $rc
for B in 10000 25000 50000 100000; do
  for M in direct localize; do
    if [ $M = direct ]; then E="WH_LINEAR_DIRECT_NNZ=100000000"; else E="WH_LINEAR_STEP=localize"; fi
    timeout -k 10 300 env $E python bench.py --model linear --batch $B > $OUT/lin_${M}_$B.log 2>&1 || exit $?
    echo "$B $M $(tail -1 $OUT/lin_${M}_$B.log | cut -c95-150)"
  done
done
for B in 10000 100000; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d $OUT/prof_$B -o run -- python3 bench.py --model linear --batch $B --steps 100 --warmup 5 > $OUT/prof_$B.log 2>&1 || exit $?
  WH_LINEAR_DIRECT_NNZ=100000000 timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d $OUT/profd_$B -o run -- python3 bench.py --model linear --batch $B --steps 100 --warmup 5 > $OUT/profd_$B.log 2>&1 || exit $?
done
for d in prof_10000 profd_10000 prof_100000 profd_100000; do
  python tools/prof_summary.py $(find $OUT/$d -name '*.db' | head -1) --last-steps 50 --step-kernel k_lin_fwd > $OUT/$d.txt 2>&1 || true
  echo "== $d"; head -14 $OUT/$d.txt; tail -2 $OUT/$d.txt
done
timeout -k 10 600 python benchmarks/bench_gbdt.py --trees 20 > $OUT/gbdt.log 2>&1 || exit $?
tail -1 $OUT/gbdt.log | cut -c1-200
echo done
