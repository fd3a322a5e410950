#!/bin/bash
# One box: read-mostly tag sweep (once per 255 opens): tests, linear P = 1 / loopback 8
# interleaved, DiFacto loopback 8, kernel
# durations (k_ps_sweep_tags).
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r6e; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10 300"
$T python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_psx.py tests/test_kv_exchange.py tests/test_deterministic_gpu.py tests/test_apps_gpu.py > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
b() { $T python bench.py "$@" > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; return 1; }; tail -1 $OUT/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.2f M ex/s %.1f us/step' % (d['value']/1e6, 1000*d['ms_per_step']))"; }
for i in 1 2 3; do
  r=$(b --model linear --loopback 8) || exit 1; echo "lin_lb8 $r"
  r=$(b --model linear) || exit 1; echo "lin_p1 $r"
done | tee $OUT/ab.txt || exit 1
r=$(b --loopback 8) || exit 1; echo "dif_lb8 $r" | tee -a $OUT/ab.txt
r=$(b) || exit 1; echo "p1 $r" | tee -a $OUT/ab.txt
for m in lb8; do
  a=""; [ $m = lb8 ] && a="--loopback 8"
  $T rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$m -o run -- python bench.py --model linear $a --steps 200 > $OUT/$m.log 2>&1 || { tail -5 $OUT/$m.log; exit 1; }
done
grep -h sweep_tags $OUT/lb8/*/*kernel_stats.csv $OUT/lb8/*kernel_stats.csv 2>/dev/null | cut -c1-200 | tee -a $OUT/ab.txt || true
echo all done
