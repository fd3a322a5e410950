#!/bin/bash
# One box: AUC tests (kept-range buckets, LDS-staged count), P = 1 bench, kernel stats.
set -o pipefail
OUT=gpurun_out/r4v; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10"
$T 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "auc" > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
b() { $T 300 python bench.py "$@" 2>&1 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.2f M ex/s %.1f us/step' % (d['value']/1e6, 1000*d['ms_per_step']))"; }
for i in 1 2 3; do echo "p1 $(b)" || exit 1; done | tee $OUT/ab.txt || exit 1
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 50 --warmup 5 > $OUT/prof.log 2>&1 || exit 1
echo all done
