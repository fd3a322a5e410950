#!/bin/bash
# One box: localize partitions bounded by non-zeros (<= 16K each): tests,
# microbench on synthetic and bench_e2e text, P = 1 bench, end to end.
set -o pipefail
OUT=gpurun_out/r5a; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10 300"
$T python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_psx.py tests/test_kv_exchange.py tests/test_apps_gpu.py > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
python - <<'PY'
import sys; sys.path.insert(0, "benchmarks")
from bench_e2e import criteo_text
open("/tmp/e2e_sample.txt", "wb").write(criteo_text(450000, 100))
PY
WH_LOC_TIMING=1 $T python benchmarks/bench_localize.py > $OUT/synth.txt 2>&1 || exit 1
WH_LOC_TIMING=1 TEXT=/tmp/e2e_sample.txt $T python benchmarks/bench_localize.py > $OUT/text.txt 2>&1 || exit 1
grep -h bench $OUT/synth.txt $OUT/text.txt
b() { $T python bench.py "$@" 2>&1 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.2f M ex/s %.1f us/step' % (d['value']/1e6, 1000*d['ms_per_step']))"; }
for i in 1 2; do echo "p1 $(b)" || exit 1; echo "lb8 $(b --loopback 8)" || exit 1; done | tee $OUT/ab.txt || exit 1
ROWS=20000000 bash tools/gpu/e2e_variants.sh r5a/e2e "dif|WH_X=0|--model difacto" "lin|WH_X=0|--model linear" "difcrb|WH_X=0|--model difacto --format crb" "dif2|WH_X=0|--model difacto" || exit 1
echo all done
