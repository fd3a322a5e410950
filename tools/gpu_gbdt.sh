set -o pipefail
OUT=gpurun_out/gbdt2; mkdir -p $OUT
timeout -k 10 600 python -m pytest tests -m gpu -q -x -k "gbdt or xgboost or kmeans" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 600 python benchmarks/bench_gbdt.py --rows 11000000 --features 28 --depth 8 --trees 20 > $OUT/gbdt.log 2>&1 || { tail -30 $OUT/gbdt.log; exit 1; }
tail -1 $OUT/gbdt.log
timeout -k 10 600 python benchmarks/bench_kmeans.py --rows 10000000 --dim 128 --k 1000 > $OUT/kmeans.log 2>&1 || exit 1
tail -1 $OUT/kmeans.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 benchmarks/bench_gbdt.py --rows 11000000 --features 28 --depth 8 --trees 5 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
echo done
