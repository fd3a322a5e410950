#!/bin/bash
# linear demo under step / ingest modes, then the whole GPU suite (no -x)
set -o pipefail
OUT=gpurun_out/r3b_diag
mkdir -p $OUT
timeout -k 10 600 python -u tools/gpu/demo_modes.py linear > $OUT/demo_modes.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -15 $OUT/pytest.log
exit $rc
