#!/bin/bash
# Save the working tree's current _hip.so build as variant NAME (ab/NAME/_hip.so)
# for a same-box A/B: bash tools/gpu/run.sh TAG 2 "base|WH_AB_HIP=ab/base/_hip.so|" \
#   "NAME|WH_AB_HIP=ab/NAME/_hip.so|" ...
set -e
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
(cd "$ROOT" && python build_native.py > /dev/null)
mkdir -p "$ROOT/ab/$1"
cp "$ROOT/wormhole_amd/_hip.so" "$ROOT/ab/$1/_hip.so"
echo "ab/$1/_hip.so"
