#!/bin/bash
# One GPU-box pass: gpu tests, smoke, 1-GPU bench, kernel-trace profile.
# Usage (from repo root): bash tools/gpu_check.sh <tag>
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 python -u -m pytest tests -m gpu ${PYTEST_X--x} -q -rf --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $OUT/pytest.log
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || exit $?
tail -1 $OUT/bench.log
timeout -k 10 300 python bench.py --model linear > $OUT/bench_linear.log 2>&1 || exit $?
tail -1 $OUT/bench_linear.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 10 --warmup 3 > $OUT/prof.log 2>&1 || exit $?
echo done
