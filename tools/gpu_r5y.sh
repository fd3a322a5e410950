#!/bin/bash
# One box: localize tiles down to 1024 non-zeros for >= 256 tiles (WH_LOC_MIN_TILES):
# localize/psx tests, linear loopback 8 A/B, DiFacto P = 1 and loopback 8.
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5y; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10 300"
$T python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_psx.py tests/test_kv_exchange.py tests/test_deterministic_gpu.py tests/test_apps_gpu.py > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
b() { $T python bench.py "$@" > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; return 1; }; tail -1 $OUT/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.2f M ex/s %.1f us/step' % (d['value']/1e6, 1000*d['ms_per_step']))"; }
for i in 1 2 3; do
  r=$(b --model linear --loopback 8) || exit 1; echo "lin_lb8 tiles256 $r"
  r=$(WH_LOC_MIN_TILES=1 b --model linear --loopback 8) || exit 1; echo "lin_lb8 tiles1 $r"
done | tee $OUT/ab.txt || exit 1
r=$(b --model linear --loopback 8 --loopback-rccl) || exit 1; echo "lin_lb8_rccl tiles256 $r" | tee -a $OUT/ab.txt
r=$(b) || exit 1; echo "p1 $r" | tee -a $OUT/ab.txt
r=$(b --loopback 8) || exit 1; echo "dif_lb8 $r" | tee -a $OUT/ab.txt
WH_LOC_TIMING=0 $T python benchmarks/bench_localize.py 2>&1 | grep bench | tee -a $OUT/ab.txt
$T rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/lb8 -o run -- python bench.py --model linear --loopback 8 --steps 200 > $OUT/lb8.log 2>&1 || { tail -5 $OUT/lb8.log; exit 1; }
python tools/step_timeline.py $OUT/lb8 k_synth_criteo 5 > $OUT/lb8_timeline.txt
tail -12 $OUT/lb8_timeline.txt | cut -c1-100
echo all done
