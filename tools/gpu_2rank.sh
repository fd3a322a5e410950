#!/bin/bash
# Rehearse the multi-rank GPU code paths on a 1-GPU box: RCCL refuses two
# ranks on one device, so the ranks share GPU 0 and exchange through gloo
# (WH_COMM_BACKEND=gloo stages tensors through host memory; timings are NOT
# representative of xGMI, correctness is).  Usage: bash tools/gpu_2rank.sh TAG [NPROC...]
set -o pipefail
OUT=gpurun_out/${1:-two}
shift
NPS=${@:-2}
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests/test_kv_exchange.py -q -x -m gpu --timeout 120 --timeout-method thread > $OUT/test.log 2>&1 || { tail -40 $OUT/test.log; exit 1; }
tail -2 $OUT/test.log
for NP in $NPS; do
  for M in difacto linear; do
    WH_BENCH_SAME_GPU=1 WH_COMM_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $NP \
      --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus $NP --steps 5 --warmup 2 --prewarm 0 --model $M --batch 20000 $BENCH_EXTRA > $OUT/bench$NP.$M.log 2>&1 || { tail -40 $OUT/bench$NP.$M.log; exit 1; }
    echo "np=$NP $M: $(tail -1 $OUT/bench$NP.$M.log | cut -c1-200)"
  done
done
