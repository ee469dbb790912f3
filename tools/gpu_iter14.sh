set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_lbvh.py -q -x -p no:cacheprovider > gpurun_out/lbvh.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/sp.json 2>> gpurun_out/err.log || exit 1
