#!/bin/bash
# One box: psx stream topologies (one / two / multi) for linear and DiFacto
# over the identity and RCCL loopbacks; psx GPU tests in two-stream mode.
set -o pipefail
OUT=gpurun_out/r4w; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10"
WH_PSX_STREAMS=two $T 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_psx.py > $OUT/pytest_two.txt 2>&1 || { tail -30 $OUT/pytest_two.txt; exit 1; }
tail -1 $OUT/pytest_two.txt
b() { $T 300 python bench.py "$@" 2>&1 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.2f M ex/s %.1f us/step' % (d['value']/1e6, 1000*d['ms_per_step']))"; }
for i in 1 2; do
  for m in one two multi; do
    echo "lin_lb8_$m $(WH_PSX_STREAMS=$m b --model linear --loopback 8)" || exit 1
  done
  echo "lin_rccl_two $(WH_PSX_STREAMS=two b --model linear --loopback 8 --loopback-rccl)" || exit 1
  echo "lin_rccl_one $(WH_PSX_STREAMS=one b --model linear --loopback 8 --loopback-rccl)" || exit 1
  echo "dif_lb8_multi $(WH_PSX_STREAMS=multi b --loopback 8)" || exit 1
  echo "dif_lb8_two $(WH_PSX_STREAMS=two b --loopback 8)" || exit 1
  echo "dif_rccl_py $(b --loopback 8 --loopback-rccl)" || exit 1
  echo "dif_rccl_nat_two $(WH_PSX_NATIVE=1 WH_PSX_STREAMS=two b --loopback 8 --loopback-rccl)" || exit 1
  echo "dif_rccl_nat_multi $(WH_PSX_NATIVE=1 WH_PSX_STREAMS=multi b --loopback 8 --loopback-rccl)" || exit 1
done | tee $OUT/ab.txt || exit 1
echo all done
