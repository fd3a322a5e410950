#!/bin/bash
# One box: the linear multi-shard step's count exchange C0 right behind the
# next job's histogram (WH_PSX_C0_EARLY, default on for linear) vs behind
# the open: tests, A/B at loopback 8 (local and RCCL), host split.
set -o pipefail
OUT=gpurun_out/r5u; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10 300"
$T python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_psx.py tests/test_kv_exchange.py tests/test_apps_gpu.py > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
b() { $T python bench.py "$@" > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; return 1; }; tail -1 $OUT/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.2f M ex/s %.1f us/step' % (d['value']/1e6, 1000*d['ms_per_step']))"; }
for i in 1 2 3; do
  r=$(b --model linear --loopback 8) || exit 1; echo "lin_lb8 early $r"
  r=$(WH_PSX_C0_EARLY=0 b --model linear --loopback 8) || exit 1; echo "lin_lb8 late  $r"
done | tee $OUT/ab.txt || exit 1
r=$(b --model linear --loopback 8 --loopback-rccl) || exit 1; echo "lin_lb8_rccl early $r" | tee -a $OUT/ab.txt
r=$(WH_PSX_C0_EARLY=0 b --model linear --loopback 8 --loopback-rccl) || exit 1; echo "lin_lb8_rccl late  $r" | tee -a $OUT/ab.txt
r=$(b --model linear) || exit 1; echo "lin_p1 $r" | tee -a $OUT/ab.txt
WH_STEP_TIMING=1 $T python bench.py --loopback 8 --model linear > $OUT/lin_timing.log 2>&1 || exit 1
grep "host us" $OUT/lin_timing.log | tail -1
echo all done
