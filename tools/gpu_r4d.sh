#!/bin/bash
# Round-4 pass: native psx step + new GPU tests first, then the full suite,
# same-box benches (P=1, loopback-8 native vs Python, linear 10k), sparse
# k-means at 1M x 1M, the compute-priority A/B.
set -o pipefail
OUT=gpurun_out/r4d; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10"
$T 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_psx.py tests/test_gbdt_xchg.py tests/test_kv_exchange.py tests/test_apps_gpu.py -m gpu -k "native or loopback or xchg or sharded or qregion or fixed_bytes or csr" > $OUT/new.log 2>&1; rc=$?
tail -3 $OUT/new.log
case $rc in 0|1) ;; *) exit $rc;; esac
$T 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc2=$?
tail -3 $OUT/pytest.log
case $rc2 in 0|1) ;; *) exit $rc2;; esac
b() { $T 300 python bench.py "$@" 2>&1 | tail -1 | cut -c1-230; }
for i in 1 2; do
  echo "p1 $(b)" >> $OUT/bench.txt
  echo "lb8_native $(b --loopback 8)" >> $OUT/bench.txt
  echo "lb8_python $(WH_PSX_NATIVE=0 b --loopback 8)" >> $OUT/bench.txt
  echo "lb8rccl_native $(b --loopback 8 --loopback-rccl)" >> $OUT/bench.txt
  echo "lin_p1 $(b --model linear)" >> $OUT/bench.txt
  echo "lin_lb8_native $(b --model linear --loopback 8)" >> $OUT/bench.txt
  echo "lin_lb8_python $(WH_PSX_NATIVE=0 b --model linear --loopback 8)" >> $OUT/bench.txt
done
cat $OUT/bench.txt | cut -c1-150
$T 300 python benchmarks/bench_kmeans.py --sparse 1000000 --rows 1000000 --k 100 --nnz 32 --iters 5 > $OUT/km_sparse_k100.log 2>&1 || exit $?
tail -1 $OUT/km_sparse_k100.log
$T 300 python benchmarks/bench_kmeans.py --sparse 1000000 --rows 1000000 --k 1000 --nnz 32 --iters 3 > $OUT/km_sparse_k1000.log 2>&1 || exit $?
tail -1 $OUT/km_sparse_k1000.log
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bprof -o run -- python3 bench.py --steps 100 > $OUT/bprof.log 2>&1 || exit $?
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/lbprof -o run -- python3 bench.py --steps 100 --loopback 8 > $OUT/lbprof.log 2>&1 || exit $?
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/linprof -o run -- python3 bench.py --steps 100 --loopback 8 --model linear > $OUT/linprof.log 2>&1 || exit $?
bash tools/gpu/env_ab.sh r4d/prio "WH_COMPUTE_PRIO=1" || exit $?
echo all done rc=$rc rc2=$rc2
