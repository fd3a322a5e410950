#!/bin/bash
# quick pass: selected GPU tests, then the given benches (one per argument
# string), each a bench.py argument list; prints value + ms/step.
set -o pipefail
OUT=gpurun_out/${1:-r3q}; shift
TESTS=${TESTS:-tests/test_psx.py}
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$TESTS" != "none" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
  tail -1 $OUT/tests.log
  [ $rc -le 1 ] || exit $rc
fi
i=0
for A in "$@"; do
  i=$((i+1))
  timeout -k 10 300 env $A > $OUT/b$i.log 2>&1 || { tail -20 $OUT/b$i.log; exit 1; }
  python - "$OUT/b$i.log" "$A" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
print("%-70s %7.1f M  %.3f ms  %s" % (sys.argv[2][:70], d["value"] / 1e6, d.get("ms_per_step", 0),
                                     json.dumps(d.get("wire_bytes_per_gpu_step"))[:160]))
PY
done
echo done
