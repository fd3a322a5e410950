#!/bin/bash
# Session-4 pass: GPU tests, smoke, headline bench, GBDT bench + kernel trace.
set -o pipefail
OUT=gpurun_out/r3d; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || exit $?
tail -1 $OUT/bench.log
timeout -k 10 600 python benchmarks/bench_gbdt.py --rows 11000000 --features 28 --depth 8 --trees 20 > $OUT/gbdt.log 2>&1 || exit $?
tail -1 $OUT/gbdt.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/gprof -o run -- python3 benchmarks/bench_gbdt.py --rows 11000000 --features 28 --depth 8 --trees 20 > $OUT/gprof.log 2>&1 || exit $?
echo all done
