#!/bin/bash
set -o pipefail
bash tools/gpu/env_ab.sh ${1:-auc}_d WH_AUC_LATE=1 --steps 200 --warmup 20 || exit 1
