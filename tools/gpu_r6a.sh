#!/bin/bash
# One box: ps_open outputs as dtype views of one allocation: tests, linear lb8 throughput and host split, DiFacto P = 1 and loopback 8.
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r6a; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10 300"
$T python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_psx.py tests/test_kv_exchange.py tests/test_deterministic_gpu.py tests/test_apps_gpu.py > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
b() { $T python bench.py "$@" > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; return 1; }; tail -1 $OUT/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.2f M ex/s %.1f us/step' % (d['value']/1e6, 1000*d['ms_per_step']))"; }
for i in 1 2 3; do
  r=$(b --model linear --loopback 8) || exit 1; echo "lin_lb8 $r"
done | tee $OUT/ab.txt || exit 1
WH_STEP_TIMING=1 $T python bench.py --loopback 8 --model linear > $OUT/lin_timing.log 2>&1 || exit 1
grep "host us" $OUT/lin_timing.log | tail -1 | tee -a $OUT/ab.txt
r=$(b --model linear --loopback 8 --loopback-rccl) || exit 1; echo "lin_lb8_rccl $r" | tee -a $OUT/ab.txt
r=$(b) || exit 1; echo "p1 $r" | tee -a $OUT/ab.txt
r=$(b --loopback 8) || exit 1; echo "dif_lb8 $r" | tee -a $OUT/ab.txt
WH_LOC_TIMING=0 $T python benchmarks/bench_localize.py 2>&1 | grep bench | tee -a $OUT/ab.txt
echo all done
