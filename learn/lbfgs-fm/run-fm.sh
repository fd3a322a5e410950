#!/bin/bash
# L-BFGS factorization machine on agaricus with k ranks, then prediction
# (reference learn/lbfgs-fm/run-fm.sh). Usage: run-fm.sh nprocess
if [[ $# -lt 1 ]]; then echo "Usage: nprocess"; exit 1; fi
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
rm -rf ./*.model
"$ROOT/tracker/dmlc_local.py" -n "$1" "$ROOT/bin/fm.dmlc" "$ROOT/learn/data/agaricus.txt.train" reg_L1=1
echo "train done"
"$ROOT/bin/fm.dmlc" "$ROOT/learn/data/agaricus.txt.test" task=pred model_in=final.model
