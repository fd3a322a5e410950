set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6k; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_VALU_MFMA_COEXEC_CYCLES SQ_LDS_DATA_FIFO_FULL"
for v in "pipe|1" "base|0"; do
  IFS='|' read -r n e <<< "$v"
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 120 env WH_TMP_KM_PIPE=$e rocprofv3 --pmc $P --kernel-trace --output-format csv -d $O/${n}_p$i -o run -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_kmeans.py --iters 1 --warmup 1 > $O/${n}_p$i.log 2>&1 || { tail -20 $O/${n}_p$i.log; exit 1; }
    python3 $GRAFT_REPO_ROOT/tools/pmc_kernel.py $O/${n}_p$i k_assign_x3
  done
done
