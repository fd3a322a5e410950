#!/bin/bash
# A/B list: each argument "ENV=.. ENV2=.. | bench args"; prints value, ms/step, retries
set -o pipefail
OUT=gpurun_out/${1:-r3ab}; shift
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for A in "$@"; do
  i=$((i+1))
  E=${A%%|*}; B=${A#*|}
  timeout -k 10 300 env $E python bench.py $B > $OUT/b$i.log 2>&1 || { tail -20 $OUT/b$i.log; exit 1; }
  python - "$OUT/b$i.log" "$A" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
print("%-64s %7.1f M  %.3f ms  retries %s" % (sys.argv[2][:64], d["value"] / 1e6, d["ms_per_step"], d.get("localize_retries")))
PY
done
echo done
