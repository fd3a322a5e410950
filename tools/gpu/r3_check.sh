#!/bin/bash
# Round-3 GPU pass: gpu tests, smoke, 1-GPU benches, RCCL-loopback CU-reserve sweep.
set -o pipefail
OUT=gpurun_out/${1:-r3}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || exit $?
tail -1 $OUT/bench.log | cut -c1-400
timeout -k 10 300 python bench.py --model linear > $OUT/bench_linear.log 2>&1 || exit $?
tail -1 $OUT/bench_linear.log | cut -c1-400
timeout -k 10 300 python bench.py --model linear --batch 100000 > $OUT/bench_linear100k.log 2>&1 || exit $?
tail -1 $OUT/bench_linear100k.log | cut -c1-300
timeout -k 10 300 python bench.py --loopback 8 > $OUT/lb8.log 2>&1 || exit $?
tail -1 $OUT/lb8.log | cut -c1-300
for R in 0 16 32 64; do
  WH_RCCL_CU_RESERVE=$R timeout -k 10 300 python bench.py --loopback 8 --loopback-rccl > $OUT/lb8r_$R.log 2>&1 || exit $?
  echo "reserve $R: $(tail -1 $OUT/lb8r_$R.log | cut -c1-200)"
done
WH_COMM_TIMING=1 timeout -k 10 300 python bench.py --loopback 8 --loopback-rccl --steps 50 > $OUT/lb8r_timing.log 2>&1 || exit $?
tail -1 $OUT/lb8r_timing.log | grep -o '"wire_bytes_per_gpu_step.*'
echo done
