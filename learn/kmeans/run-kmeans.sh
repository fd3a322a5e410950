#!/bin/bash
# spherical k-means on agaricus with k ranks: <nprocess> <num_cluster> <max_iter>
# (reference learn/kmeans/kmeans.cc usage; writes the centroids to kmeans.txt)
if [[ $# -lt 3 ]]; then echo "Usage: nprocess num_cluster max_iter"; exit 1; fi
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
"$ROOT/tracker/dmlc_local.py" -n "$1" "$ROOT/bin/kmeans.dmlc" "$ROOT/learn/data/agaricus.txt.train" "$2" "$3" kmeans.txt
