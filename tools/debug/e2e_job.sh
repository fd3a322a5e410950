#!/bin/bash
# one linear.dmlc job over generated Criteo files with stack dumps on a stall
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out /tmp/ej/data
python3 - <<'PY'
import sys
sys.path.insert(0, "benchmarks")
from bench_e2e import criteo_text
for i in range(4):
    open("/tmp/ej/data/train-part_%d.txt" % i, "wb").write(criteo_text(500000, 100 + i))
open("/tmp/ej/job.conf", "w").write('train_data = "/tmp/ej/data/"\ndata_format = "criteo"\nminibatch = 100000\nmax_data_pass = 1\nprint_sec = 1\nlambda_l1 = 4\nlr_eta = 0.1\n')
PY
cd /tmp/ej
WH_HANG_DUMP=20 timeout -k 10 90 python3 "$GRAFT_REPO_ROOT/tracker/dmlc_local.py" -n 1 -s 1 "$GRAFT_REPO_ROOT/bin/linear.dmlc" job.conf > "$GRAFT_REPO_ROOT/gpurun_out/ej.log" 2>&1
echo "exit $?" >> "$GRAFT_REPO_ROOT/gpurun_out/ej.log"
