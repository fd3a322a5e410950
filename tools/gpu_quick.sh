#!/bin/bash
# GPU tests + 1-GPU bench + rocprof kernel trace of the headline bench.
set -o pipefail
OUT=gpurun_out/${1:-quick}
mkdir -p $OUT
timeout -k 10 900 python -m pytest tests -m gpu -q -x > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python bench.py --steps 100 --warmup 10 > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 20 --warmup 5 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
echo done
