#!/bin/bash
# PMC counter passes over the 1-GPU bench (each pass in its own rocprofv3 run,
# kernel-trace only alongside the counters). Usage: bash tools/gpu_pmc.sh <tag> [bench args]
set -o pipefail
TAG=${1:-pmc}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ARGS=${@:---steps 3 --warmup 2}
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_ATOMIC_sum --kernel-trace --output-format csv -d $OUT/p1 -o run -- python3 bench.py $ARGS > $OUT/p1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/p2 -o run -- python3 bench.py $ARGS > $OUT/p2.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/p3 -o run -- python3 bench.py $ARGS > $OUT/p3.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d $OUT/p4 -o run -- python3 bench.py $ARGS > $OUT/p4.log 2>&1 || exit $?
echo pmc done
