set -o pipefail
bash tools/gpu_2rank.sh two || exit 1
timeout -k 10 300 python bench.py > gpurun_out/two/bench1.log 2>&1 || exit 1
tail -1 gpurun_out/two/bench1.log
