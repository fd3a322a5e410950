#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u benchmarks/bench_gbdt.py --trees 20 > gpurun_out/gbdt.tmp 2>&1 || { echo GBDT FAILED; tail -30 gpurun_out/gbdt.tmp; exit 1; }
grep '^{' gpurun_out/gbdt.tmp
WH_HOST_PROFILE=1 timeout -k 10 300 python -u -c "
import cProfile, pstats, sys
sys.argv=['bench_gbdt.py','--trees','10']
sys.path.insert(0,'benchmarks')
import bench_gbdt
cProfile.run('bench_gbdt.main()', 'gpurun_out/gbdt.prof')
p = pstats.Stats('gpurun_out/gbdt.prof'); p.sort_stats('tottime').print_stats(25)
" > gpurun_out/gbdt_host.txt 2>&1 || { echo HOSTPROF FAILED; tail -20 gpurun_out/gbdt_host.txt; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/gb -o gb -- python3 benchmarks/bench_gbdt.py --trees 6 > gpurun_out/prof/gb.log 2>&1 || { echo PROF FAILED; tail -20 gpurun_out/prof/gb.log; exit 1; }
