#!/bin/bash
# new GPU tests, then A/B: DiFacto direct pull vs copy, linear fused vs three kernels
set -o pipefail
OUT=gpurun_out/r3b_ab2
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_apps_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
bash tools/gpu/env_ab.sh r3b_ab2/difacto "WH_DIFACTO_PULL=copy" || exit $?
bash tools/gpu/env_ab.sh r3b_ab2/linear "WH_LINEAR_FUSED=0" --model linear || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 10 --warmup 3 > $OUT/prof.log 2>&1 || exit $?
