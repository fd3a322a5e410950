#!/bin/bash
# tests + smoke + benches (DiFacto, linear fused / unfused A/B) + linear kernel trace
set -o pipefail
TAG=${1:-r3b}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
for i in 1 2; do
timeout -k 10 300 python bench.py --model linear > $OUT/bench_linear_$i.log 2>&1 || exit $?
tail -1 $OUT/bench_linear_$i.log | cut -c1-200
WH_LINEAR_FUSED=0 timeout -k 10 300 python bench.py --model linear > $OUT/bench_linear_unfused_$i.log 2>&1 || exit $?
tail -1 $OUT/bench_linear_unfused_$i.log | cut -c1-200
done
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || exit $?
tail -1 $OUT/bench.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_lin -o run -- python3 bench.py --model linear --steps 200 --warmup 20 > $OUT/prof_lin.log 2>&1 || exit $?
echo done
exit $rc
