#!/bin/bash
# Kernel-trace profiles of the multi-shard step (identity and RCCL loopback),
# linear multi-shard throughput, host profile of the RCCL loopback step.
set -o pipefail
OUT=gpurun_out/${1:-r3p}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_psx.py -m gpu -q --timeout 120 --timeout-method thread > $OUT/psx_tests.log 2>&1; rc=$?
tail -1 $OUT/psx_tests.log
[ $rc -le 1 ] || exit $rc
for BPC in 4 6 8; do
  WH_FM_BLOCKS_PER_CU=$BPC timeout -k 10 300 python bench.py > $OUT/bpc_$BPC.log 2>&1 || exit $?
  echo "fm blocks/CU $BPC: $(tail -1 $OUT/bpc_$BPC.log | cut -c100-160)"
done
for B in 10000 100000; do
  timeout -k 10 300 python bench.py --model linear --batch $B > $OUT/lin_p1_$B.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --model linear --batch $B --loopback 8 > $OUT/lin_lb8_$B.log 2>&1 || exit $?
  echo "linear $B: P1 $(tail -1 $OUT/lin_p1_$B.log | cut -c100-160) lb8 $(tail -1 $OUT/lin_lb8_$B.log | cut -c100-160)"
done
WH_HOST_PROFILE=$OUT/host_lin10k timeout -k 10 300 python bench.py --model linear --steps 300 > $OUT/lin10k_host.log 2>&1 || exit $?
WH_HOST_PROFILE=$OUT/host_lb8r timeout -k 10 300 python bench.py --loopback 8 --loopback-rccl --steps 100 > $OUT/lb8r_host.log 2>&1 || exit $?
tail -1 $OUT/lb8r_host.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d $OUT/prof_lb8r -o run -- python3 bench.py --loopback 8 --loopback-rccl --steps 100 --warmup 5 > $OUT/prof_lb8r.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d $OUT/prof_lb8 -o run -- python3 bench.py --loopback 8 --steps 100 --warmup 5 > $OUT/prof_lb8.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d $OUT/prof_lin10k -o run -- python3 bench.py --model linear --steps 100 --warmup 5 > $OUT/prof_lin10k.log 2>&1 || exit $?
for d in prof_lb8r prof_lb8 prof_lin10k; do
  db=$(find $OUT/$d -name '*.db' | head -1)
  python tools/prof_summary.py $db --last-steps 50 > $OUT/$d.txt 2>&1 || true
  head -3 $OUT/$d.txt
done
echo done
