set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_bvh_exact.py -q -s -p no:cacheprovider > gpurun_out/bvh.log 2>&1
timeout -k 10 600 python bench.py --spp 4 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err
