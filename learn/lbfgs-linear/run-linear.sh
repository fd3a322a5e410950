#!/bin/bash
# L-BFGS logistic regression on agaricus with k ranks, then prediction
# (reference learn/lbfgs-linear/run-linear.sh). Usage: run-linear.sh nprocess
if [[ $# -lt 1 ]]; then echo "Usage: nprocess"; exit 1; fi
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
rm -rf ./*.model
# the program splits the input over the ranks itself
"$ROOT/tracker/dmlc_local.py" -n "$1" "$ROOT/bin/lbfgs.dmlc" "$ROOT/learn/data/agaricus.txt.train" reg_L1=1
"$ROOT/bin/lbfgs.dmlc" "$ROOT/learn/data/agaricus.txt.test" task=pred model_in=final.model
