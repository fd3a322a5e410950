#!/bin/bash
# Round-4 first pass: full GPU suite (no -x: see every failure), smoke,
# headline bench, GBDT 500 trees + kernel trace.
set -o pipefail
OUT=gpurun_out/r4a; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -5 $OUT/pytest.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || exit $?
tail -1 $OUT/bench.log
timeout -k 10 600 python benchmarks/bench_gbdt.py --trees 500 > $OUT/gbdt.log 2>&1 || exit $?
tail -1 $OUT/gbdt.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/gprof -o run -- python3 benchmarks/bench_gbdt.py --trees 100 > $OUT/gprof.log 2>&1 || exit $?
echo all done rc=$rc
