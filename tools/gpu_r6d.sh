#!/bin/bash
# One box: linear forward with every local id of a pass loaded before the
# weight gathers: tests, linear P = 1 / loopback 8 interleaved, kernel
# durations of k_lin_fwd in both steps.
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r6d; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10 300"
$T python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_psx.py tests/test_kv_exchange.py tests/test_deterministic_gpu.py tests/test_apps_gpu.py > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
b() { $T python bench.py "$@" > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; return 1; }; tail -1 $OUT/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.2f M ex/s %.1f us/step' % (d['value']/1e6, 1000*d['ms_per_step']))"; }
for i in 1 2 3; do
  r=$(b --model linear --loopback 8) || exit 1; echo "lin_lb8 $r"
  r=$(b --model linear) || exit 1; echo "lin_p1 $r"
done | tee $OUT/ab.txt || exit 1
for m in lb8 p1; do
  a=""; [ $m = lb8 ] && a="--loopback 8"
  $T rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$m -o run -- python bench.py --model linear $a --steps 200 > $OUT/$m.log 2>&1 || { tail -5 $OUT/$m.log; exit 1; }
done
python - <<'PY' | tee -a $OUT/ab.txt
import csv, glob, collections, os
out = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/r6d"
for m in ("lb8", "p1"):
    path = glob.glob(out + "/" + m + "/**/*kernel_trace.csv", recursive=True)[0]
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        d[r["Kernel_Name"].split("(")[0][-40:]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:10]:
        v = sorted(v)
        print("%s %-40s n=%d median %.1f us" % (m, k, len(v), v[len(v) // 2]))
PY
echo all done
