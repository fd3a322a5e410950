#!/bin/bash
# Local CI gate: build everything for gfx950, then the CPU test tier.
# The GPU tier: bash tools/gpu_check.sh <tag> on an MI355X box.
set -euo pipefail
cd "$(dirname "$0")/.."
python build_native.py -j "${JOBS:-8}"
python -c "import __graft_entry__ as g; g.build()"
python -m pytest tests/ -x -q -m "not gpu" -n "${PYTEST_WORKERS:-4}"
