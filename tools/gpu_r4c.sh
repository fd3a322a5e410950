#!/bin/bash
# Round-4 pass 3: new GPU tests, then the full suite, sparse k-means at 1M x 1M,
# GBDT feature-sharded rehearsal.
set -o pipefail
OUT=gpurun_out/r4c; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10"
$T 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gbdt_xchg.py tests/test_kv_exchange.py tests/test_apps_gpu.py -m gpu -k "xchg or sharded or qregion or fixed_bytes or csr" > $OUT/new.log 2>&1; rc=$?
tail -3 $OUT/new.log
case $rc in 0|1) ;; *) exit $rc;; esac
$T 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc2=$?
tail -3 $OUT/pytest.log
case $rc2 in 0|1) ;; *) exit $rc2;; esac
$T 300 python benchmarks/bench_kmeans.py --sparse 1000000 --rows 1000000 --k 100 --nnz 32 --iters 5 > $OUT/km_sparse_k100.log 2>&1 || exit $?
tail -1 $OUT/km_sparse_k100.log
$T 300 python benchmarks/bench_kmeans.py --sparse 1000000 --rows 1000000 --k 1000 --nnz 32 --iters 3 > $OUT/km_sparse_k1000.log 2>&1 || exit $?
tail -1 $OUT/km_sparse_k1000.log
$T 300 python benchmarks/bench_kmeans.py > $OUT/km_dense.log 2>&1 || exit $?
tail -1 $OUT/km_dense.log
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kprof -o run -- python3 benchmarks/bench_kmeans.py --sparse 1000000 --rows 1000000 --k 1000 --nnz 32 --iters 3 > $OUT/kprof.log 2>&1 || exit $?
for i in 1 2; do $T 300 python bench.py > $OUT/bench$i.log 2>&1 || exit $?; tail -1 $OUT/bench$i.log | cut -c1-200; done
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bprof -o run -- python3 bench.py --steps 100 > $OUT/bprof.log 2>&1 || exit $?
bash tools/gpu/env_ab.sh r4c/prio "WH_COMPUTE_PRIO=1" || exit $?
echo all done rc=$rc rc2=$rc2
