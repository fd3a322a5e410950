#!/bin/bash
# One box: localize microbenchmark on bench_e2e.py's Criteo text vs the
# synthetic generator, with per-partition dedup phase timings.
set -o pipefail
OUT=gpurun_out/r4z; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
python - <<'PY'
import sys; sys.path.insert(0, "benchmarks")
from bench_e2e import criteo_text
open("/tmp/e2e_sample.txt", "wb").write(criteo_text(450000, 100))
PY
T="timeout -k 10 300"
WH_LOC_TIMING=1 $T python benchmarks/bench_localize.py > $OUT/synth.txt 2>&1 || exit 1
WH_LOC_TIMING=1 TEXT=/tmp/e2e_sample.txt $T python benchmarks/bench_localize.py > $OUT/text.txt 2>&1 || exit 1
TEXT=/tmp/e2e_sample.txt $T rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 benchmarks/bench_localize.py > $OUT/kt.txt 2>&1 || exit 1
cat $OUT/synth.txt $OUT/text.txt
echo all done
