#!/bin/bash
# One box: psx / guard GPU tests, the linear multi-shard step's host trims
# (loopback C0 fill, store summary every 4 opens) A/B, and a host API trace.
set -o pipefail
OUT=gpurun_out/r4r; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10"
$T 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_psx.py tests/test_kv_exchange.py tests/test_store_guard.py > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
b() { $T 300 python bench.py "$@" 2>&1 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.2f M ex/s %.1f us/step' % (d['value']/1e6, 1000*d['ms_per_step']))"; }
for i in 1 2; do
  echo "lin_p1 $(b --model linear)" || exit 1
  echo "lin_lb8 $(b --model linear --loopback 8)" || exit 1
  echo "lin_lb8_guard1 $(WH_GUARD_EVERY=1 b --model linear --loopback 8)" || exit 1
  echo "lin_rccl $(b --model linear --loopback 8 --loopback-rccl)" || exit 1
  echo "dif_lb8 $(b --loopback 8)" || exit 1
done | tee $OUT/ab.txt || exit 1
WH_STEP_TIMING=1 $T 300 python bench.py --loopback 8 --model linear > $OUT/lin_timing.log 2>&1 || exit 1
grep "host us" $OUT/lin_timing.log | tail -1
$T 300 rocprofv3 --hip-trace --kernel-trace --stats -d $OUT/ht -o run --output-format csv -- python bench.py --model linear --loopback 8 --steps 60 --warmup 20 > $OUT/ht.log 2>&1 || exit 1
echo all done
