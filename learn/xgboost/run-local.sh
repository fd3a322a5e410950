#!/bin/bash
# distributed GBDT on agaricus with k ranks, then prediction and a text dump
# with the feature map (local analogue of reference learn/xgboost/run_yarn.sh).
# Outputs land in the current directory. Usage: run-local.sh nworkers
if [[ $# -lt 1 ]]; then echo "Usage: nworkers"; exit 1; fi
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
OUT=$(pwd)
D="$ROOT/learn/data"
CONF="$ROOT/learn/xgboost/mushroom.conf"
"$ROOT/tracker/dmlc_local.py" -n "$1" "$ROOT/bin/xgboost.dmlc" "$CONF" data="$D/agaricus.txt.train" \
    "eval[test]=$D/agaricus.txt.test" model_out="$OUT/mushroom.final.model"
"$ROOT/bin/xgboost.dmlc" "$CONF" task=pred model_in="$OUT/mushroom.final.model" \
    test:data="$D/agaricus.txt.test" name_pred="$OUT/pred.txt"
"$ROOT/bin/xgboost.dmlc" "$CONF" task=dump model_in="$OUT/mushroom.final.model" \
    fmap="$D/featmap.txt" name_dump="$OUT/dump.nice.txt"
