#!/bin/bash
# PMC counter passes over any python program (each pass its own rocprofv3 run,
# kernel-trace only alongside the counters).
# Usage: bash tools/gpu_pmc2.sh <tag> <script.py> [args...]
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
P="timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv"
$P --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_ATOMIC_sum -d $OUT/p1 -o run -- python3 "$@" > $OUT/p1.log 2>&1 || exit $?
$P --pmc FETCH_SIZE -d $OUT/p2 -o run -- python3 "$@" > $OUT/p2.log 2>&1 || exit $?
$P --pmc WRITE_SIZE -d $OUT/p3 -o run -- python3 "$@" > $OUT/p3.log 2>&1 || exit $?
$P --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d $OUT/p4 -o run -- python3 "$@" > $OUT/p4.log 2>&1 || exit $?
echo pmc $TAG done
