#!/bin/bash
# One box: kernel trace of the end-to-end DiFacto run from Criteo text
# (ingest kernels vs training kernels on the one GPU).
set -o pipefail
OUT=gpurun_out/r4x; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
W=/tmp/wh_e2e_x
timeout -k 10 400 python benchmarks/bench_e2e.py --rows 10000000 --files 4 --dir $W --model difacto > $OUT/gen.json 2> $OUT/gen.err || { tail -20 $OUT/gen.err; exit 1; }
tail -1 $OUT/gen.json | cut -c1-200
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/kt -o run -- python3 benchmarks/bench_e2e.py --rows 10000000 --files 4 --dir $W --reuse --model difacto > $OUT/kt.json 2> $OUT/kt.err || { tail -20 $OUT/kt.err; exit 1; }
tail -1 $OUT/kt.json | cut -c1-200
rm -rf $W
echo all done
