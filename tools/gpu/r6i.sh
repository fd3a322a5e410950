set -o pipefail
O=gpurun_out/r6i; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_difacto_native.py -x -v --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
run() { tag=$1; shift; timeout -k 10 240 env "$@" > $O/$tag.log 2>&1 || { echo "FAIL $tag"; tail -5 $O/$tag.log; exit 1; }; echo "$tag $(grep -o '"value": [0-9.e+]*' $O/$tag.log) $(grep -o '"ms_per_step": [0-9.]*' $O/$tag.log)"; grep "host us/call" $O/$tag.log | tail -1 || true; }
run nat1 python bench.py --steps 200 --warmup 20
run py1 WH_DIFACTO_NATIVE=0 python bench.py --steps 200 --warmup 20
run nat2 python bench.py --steps 200 --warmup 20
run py2 WH_DIFACTO_NATIVE=0 python bench.py --steps 200 --warmup 20
run d16nat WH_TIMING=step python bench.py --dim 16 --batch 1000 --steps 2000 --warmup 100 --prewarm 2000
run d16py WH_DIFACTO_NATIVE=0 python bench.py --dim 16 --batch 1000 --steps 2000 --warmup 100 --prewarm 2000
