#!/bin/bash
# Same-box A/B: native vs Python multi-shard step (loopback 8 / loopback-8 RCCL),
# P=1 after the lid-fold revert; the two failing GPU tests.
set -o pipefail
OUT=gpurun_out/r4e; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10"
$T 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_store_guard.py -m gpu -k "split_kernel or shrinking" > $OUT/fix.log 2>&1; rc=$?
tail -2 $OUT/fix.log
case $rc in 0|1) ;; *) exit $rc;; esac
b() { $T 300 python bench.py "$@" 2>&1 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.2f M ex/s %.1f us/step' % (d['value']/1e6, 1000*d['ms_per_step']))"; }
for i in 1 2 3; do
  echo "p1 $(b)"
  echo "lb8_native $(b --loopback 8)"
  echo "lb8_python $(WH_PSX_NATIVE=0 b --loopback 8)"
  echo "rccl_native $(b --loopback 8 --loopback-rccl)"
  echo "rccl_python $(WH_PSX_NATIVE=0 b --loopback 8 --loopback-rccl)"
done | tee $OUT/ab.txt
bash tools/gpu/env_ab.sh r4e/xcd "WH_BWD_XCD=0" || exit $?
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bprof -o run -- python3 bench.py --steps 100 > $OUT/bprof.log 2>&1 || exit $?
WH_BWD_XCD=0 $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bprof0 -o run -- python3 bench.py --steps 100 > $OUT/bprof0.log 2>&1 || exit $?
$T 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $OUT/pmc_xcd -o run -- python3 bench.py --steps 10 --warmup 2 --prewarm 100 > $OUT/pmc_xcd.log 2>&1 || exit $?
WH_BWD_XCD=0 $T 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $OUT/pmc_rr -o run -- python3 bench.py --steps 10 --warmup 2 --prewarm 100 > $OUT/pmc_rr.log 2>&1 || exit $?
echo all done rc=$rc
