set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6h; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in "base|" "noepi|WH_AB_HIP=$GRAFT_REPO_ROOT/ab/kmv1/_hip.so" "nodma|WH_AB_HIP=$GRAFT_REPO_ROOT/ab/kmv2/_hip.so"; do
  IFS='|' read -r n e <<< "$v"
  export WH_AB_HIP=; [ -n "$e" ] && export "$e"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/km_$n -o run -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_kmeans.py --iters 2 --warmup 1 > $O/km_$n.log 2>&1 || { tail -20 $O/km_$n.log; exit 1; }
  echo "== $n"; grep -h "k_assign_x3\|k_refine" $(find $O/km_$n -name "*kernel_stats.csv") | cut -d, -f1-5
done
unset WH_AB_HIP
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gbdtprof -o run -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_gbdt.py --trees 20 > $O/gbdtprof.log 2>&1 || { tail -20 $O/gbdtprof.log; exit 1; }
echo "== gbdt"; head -14 $(find $O/gbdtprof -name "*kernel_stats.csv") | cut -d, -f1-5
for v in "p1|" "lb8|--loopback 8"; do
  IFS='|' read -r n a <<< "$v"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/dif_$n -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 100 --warmup 10 --prewarm 300 $a > $O/dif_$n.log 2>&1 || { tail -20 $O/dif_$n.log; exit 1; }
  echo "== difacto $n"; head -30 $(find $O/dif_$n -name "*kernel_stats.csv") | cut -d, -f1-5
done
