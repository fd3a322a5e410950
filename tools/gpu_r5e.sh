#!/bin/bash
# One box: Criteo parser with LDS-staged lines: ingest GPU tests, parse
# kernel times (rocprofv3 stats of 50 parses of a 100k-line block).
set -o pipefail
OUT=gpurun_out/r5e; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10 300"
$T python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_ingest.py > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
cat > /tmp/parse_bench.py <<'PY'
import sys, torch
sys.path.insert(0, "benchmarks"); sys.path.insert(0, ".")
from bench_e2e import criteo_text
from wormhole_amd import _native
hip = _native.hip()
t = torch.frombuffer(bytearray(criteo_text(100000, 7)), dtype=torch.uint8).cuda()
for _ in range(5): hip.parse_criteo(t, 100000, True)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(50): hip.parse_criteo(t, 100000, True)
e1.record(); torch.cuda.synchronize()
print("parse_criteo 100k lines: %.1f us/call" % (e0.elapsed_time(e1) / 50 * 1000))
PY
$T python /tmp/parse_bench.py || exit 1
$T rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 /tmp/parse_bench.py > $OUT/kt.log 2>&1 || exit 1
echo all done
