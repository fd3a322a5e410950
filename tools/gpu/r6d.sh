set -o pipefail
O=gpurun_out/r6d; mkdir -p $O
run() { tag=$1; shift; timeout -k 10 240 env "$@" > $O/$tag.log 2>&1 || { echo "FAIL $tag"; tail -5 $O/$tag.log; exit 1; }; echo "$tag $(grep -o '"value": [0-9.e+]*' $O/$tag.log) $(grep -o '"ms_per_step": [0-9.]*' $O/$tag.log)"; }
run head1 python bench.py --steps 200 --warmup 20
run head2 python bench.py --steps 200 --warmup 20
run d16b1k WH_TIMING=step python bench.py --dim 16 --batch 1000 --steps 2000 --warmup 100 --prewarm 2000
run d16b1k_lb8 WH_TIMING=step python bench.py --dim 16 --batch 1000 --steps 2000 --warmup 100 --prewarm 2000 --loopback 8
run lin_lb8r WH_TIMING=step python bench.py --model linear --loopback 8 --loopback-rccl --steps 1000 --warmup 50
run lin_p1 WH_TIMING=step python bench.py --model linear --steps 1000 --warmup 50
run dif_lb8r python bench.py --loopback 8 --loopback-rccl --steps 200 --warmup 20
