#!/bin/bash
# Concurrent kernel trace of a bench.py configuration (rocprofv3
# --kernel-trace, launches NOT serialised) and the timeline of three steps
# near the end (tools/step_timeline.py: gap, duration, queue, idle time).
# Usage: bash tools/gpu/timeline.sh TAG NAME [bench.py args]
set -o pipefail
TAG=$1; NAME=$2; shift 2
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$NAME" -o run -- \
  python3 "$ROOT/bench.py" --steps 30 --warmup 5 --prewarm 300 "$@" > "$OUT/$NAME.log" 2>&1 || exit $?
for b in 4 3 2; do
  python3 "$ROOT/tools/step_timeline.py" "$OUT/$NAME" k_synth_criteo $b
done > "$OUT/$NAME.timeline.txt"
grep "^step" "$OUT/$NAME.timeline.txt"
