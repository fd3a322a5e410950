#!/bin/bash
set -o pipefail
bash tools/gpu/env_ab.sh ${1:-guard}_d WH_GUARD_SIDE=0 --steps 200 --warmup 20 || exit 1
bash tools/gpu/env_ab.sh ${1:-guard}_lb8 WH_GUARD_SIDE=0 --loopback 8 --steps 200 --warmup 20 || exit 1
