#!/bin/bash
# Input-pipeline stage rates (bench_ingest.py), then a kernel trace of the
# linear step at the published minibatch and the two headline benches.
set -o pipefail
OUT=gpurun_out/${1:-r3i}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u benchmarks/bench_ingest.py --crb --dir /tmp/whi_$$ > $OUT/ingest.json 2> $OUT/ingest.err || { tail -20 $OUT/ingest.err; exit 1; }
cat $OUT/ingest.json
rm -rf /tmp/whi_$$
timeout -k 10 300 python bench.py --model linear > $OUT/lin10k.log 2>&1 || { tail -20 $OUT/lin10k.log; exit 1; }
echo "linear 10k: $(tail -1 $OUT/lin10k.log | cut -c100-170)"
timeout -k 10 300 python bench.py > $OUT/difacto.log 2>&1 || { tail -20 $OUT/difacto.log; exit 1; }
echo "difacto: $(tail -1 $OUT/difacto.log | cut -c80-170)"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format rocpd -d $OUT/prof_lin10k -o run -- python3 bench.py --model linear --steps 100 --warmup 5 > $OUT/prof_lin10k.log 2>&1 || exit $?
db=$(find $OUT/prof_lin10k -name '*.db' | head -1)
python tools/prof_summary.py $db --last-steps 50 > $OUT/prof_lin10k.txt 2>&1 || true
head -30 $OUT/prof_lin10k.txt
echo done
