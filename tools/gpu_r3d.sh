#!/bin/bash
# Session-4 pass: full GPU check (tests, smoke, benches, profile), then GBDT bench + kernel trace.
set -o pipefail
bash tools/gpu_check.sh r3d || exit $?
OUT=gpurun_out/r3d; mkdir -p $OUT
timeout -k 10 600 python benchmarks/bench_gbdt.py --rows 11000000 --features 28 --depth 8 --trees 20 > $OUT/gbdt.log 2>&1 || exit $?
tail -1 $OUT/gbdt.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/gprof -o run -- python3 benchmarks/bench_gbdt.py --rows 11000000 --features 28 --depth 8 --trees 20 > $OUT/gprof.log 2>&1 || exit $?
echo all done
