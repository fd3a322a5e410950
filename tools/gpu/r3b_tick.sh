#!/bin/bash
# GPU tests, then linear (10k) and DiFacto benches + kernel stats
set -o pipefail
OUT=gpurun_out/${1:-r3b_tick}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --model linear > $OUT/lin.$i.log 2>&1 || exit $?
  echo "lin $i $(tail -1 $OUT/lin.$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,2), round(d["ms_per_step"]*1e3,1), "us", d["train_auc"])')"
  timeout -k 10 300 python bench.py > $OUT/dif.$i.log 2>&1 || exit $?
  echo "dif $i $(tail -1 $OUT/dif.$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,2), round(d["ms_per_step"]*1e3,1), "us", d["train_auc"])')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_lin -o run -- python3 bench.py --model linear > $OUT/prof_lin.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_dif -o run -- python3 bench.py --steps 10 --warmup 3 > $OUT/prof_dif.log 2>&1 || exit $?
python3 - <<'PY'
import csv,sys
out=sys.argv[1] if len(sys.argv)>1 else None
for d in ['prof_lin','prof_dif']:
    print(d)
    for r in list(csv.DictReader(open('gpurun_out/r3b_tick/%s/run_kernel_stats.csv' % d)))[:12]:
        print("  %-58s %6s %9.1f" % (r['Name'][:58], r['Calls'], float(r['AverageNs'])/1e3))
PY
