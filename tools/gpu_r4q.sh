#!/bin/bash
# One box: psx GPU tests, then the one-stream native step A/B (linear and
# DiFacto over the identity and RCCL loopbacks), then CRB vs text end to end.
set -o pipefail
OUT=gpurun_out/r4q; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10"
$T 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_psx.py tests/test_kv_exchange.py > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
b() { $T 300 python bench.py "$@" 2>&1 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.2f M ex/s %.1f us/step' % (d['value']/1e6, 1000*d['ms_per_step']))"; }
for i in 1 2; do
  echo "lin_p1 $(b --model linear)" || exit 1
  echo "lin_lb8_one $(b --model linear --loopback 8)" || exit 1
  echo "lin_lb8_multi $(WH_PSX_STREAMS=multi b --model linear --loopback 8)" || exit 1
  echo "lin_rccl_one $(b --model linear --loopback 8 --loopback-rccl)" || exit 1
  echo "lin_rccl_multi $(WH_PSX_STREAMS=multi b --model linear --loopback 8 --loopback-rccl)" || exit 1
  echo "dif_lb8_multi $(b --loopback 8)" || exit 1
  echo "dif_lb8_one $(WH_PSX_STREAMS=one b --loopback 8)" || exit 1
done | tee $OUT/ab.txt || exit 1
WH_STEP_TIMING=1 $T 300 python bench.py --loopback 8 --model linear > $OUT/lin_timing.log 2>&1 || exit 1
grep "host us" $OUT/lin_timing.log | tail -2
ROWS=20000000 bash tools/gpu/e2e_variants.sh r4q/e2e "lincrb|WH_X=0|--model linear --format crb" "difcrb|WH_X=0|--model difacto --format crb" "lin|WH_X=0|--model linear" "dif|WH_X=0|--model difacto" "lincrb2|WH_X=0|--model linear --format crb" "difcrb2|WH_X=0|--model difacto --format crb" || exit 1
echo all done
