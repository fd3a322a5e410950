#!/bin/bash
# One box: heavy-id partition count (WH_LOC_HEAVY) on the synthetic bench and
# end to end from Criteo text (whose int fields give ~200 ids above the
# heavy threshold per minibatch); dedup kernel time from a kernel trace.
set -o pipefail
OUT=gpurun_out/r4y; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T="timeout -k 10"
b() { $T 300 python bench.py "$@" 2>&1 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.2f M ex/s %.1f us/step' % (d['value']/1e6, 1000*d['ms_per_step']))"; }
for i in 1 2; do
  for h in 128 256 512; do echo "p1_heavy$h $(WH_LOC_HEAVY=$h b)" || exit 1; done
done | tee $OUT/ab.txt || exit 1
ROWS=20000000 bash tools/gpu/e2e_variants.sh r4y/e2e "dif128|WH_LOC_HEAVY=128|--model difacto" "dif256|WH_LOC_HEAVY=256|--model difacto" "dif512|WH_LOC_HEAVY=512|--model difacto" "dif128b|WH_LOC_HEAVY=128|--model difacto" "dif256b|WH_LOC_HEAVY=256|--model difacto" || exit 1
W=/tmp/wh_e2e_y
for h in 128 256; do
  $T 400 python benchmarks/bench_e2e.py --rows 4000000 --files 4 --dir $W --reuse --model difacto > /dev/null 2>&1 || exit 1
  WH_LOC_HEAVY=$h $T 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/kt$h -o run -- python3 benchmarks/bench_e2e.py --rows 4000000 --files 4 --dir $W --reuse --model difacto > $OUT/kt$h.json 2> $OUT/kt$h.err || exit 1
done
rm -rf $W
echo all done
