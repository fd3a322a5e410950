set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6j; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for n in kmv0 kmv3 kmv2; do
  timeout -k 10 300 env WH_TMP_KM_PIPE=0 WH_AB_HIP=$GRAFT_REPO_ROOT/ab/$n/_hip.so rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o run -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_kmeans.py --iters 2 --warmup 1 > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
  echo "== $n"; python3 $GRAFT_REPO_ROOT/tools/kstats.py $O/$n 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pipe -o run -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_kmeans.py --iters 2 --warmup 1 > $O/pipe.log 2>&1 || { tail -20 $O/pipe.log; exit 1; }
echo "== pipe (head build)"; python3 $GRAFT_REPO_ROOT/tools/kstats.py $O/pipe 1
