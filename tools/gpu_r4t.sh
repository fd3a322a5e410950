#!/bin/bash
# One box: the P = 1 localize side stream without its wait on the compute
# stream (default) vs with it (WH_LOC_WAIT_CUR=1); GPU tests of the learners.
set -o pipefail
OUT=gpurun_out/r4t; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10"
b() { $T 300 python bench.py "$@" 2>&1 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.2f M ex/s %.1f us/step' % (d['value']/1e6, 1000*d['ms_per_step']))"; }
for i in 1 2 3; do
  echo "p1_nowait $(b)" || exit 1
  echo "p1_wait $(WH_LOC_WAIT_CUR=1 b)" || exit 1
done | tee $OUT/ab.txt || exit 1
$T 300 rocprofv3 --kernel-trace -d $OUT/kt -o run --output-format csv -- python bench.py --steps 60 --prewarm 300 > $OUT/kt.log 2>&1 || exit 1
$T 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_apps_gpu.py tests/test_deterministic_gpu.py > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
echo all done
