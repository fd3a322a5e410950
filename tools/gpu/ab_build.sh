#!/bin/bash
# Build the committed HEAD's _hip.so into ab/base/ (the A of a same-box A/B;
# the working tree's build is the B). Usage (CPU side): bash tools/gpu/ab_build.sh
# then on the GPU: bash tools/gpu/run.sh TAG 2 "base|WH_AB_HIP=ab/base/_hip.so|" "new||"
set -e
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
W=$(mktemp -d)
git -C "$ROOT" worktree add -q --detach "$W" HEAD
(cd "$W" && python build_native.py > /dev/null)
mkdir -p "$ROOT/ab/base"
cp "$W/wormhole_amd/_hip.so" "$ROOT/ab/base/_hip.so"
git -C "$ROOT" worktree remove --force "$W"
echo "ab/base/_hip.so from $(git -C "$ROOT" log --oneline -1 | cut -c1-60)"
