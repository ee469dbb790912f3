set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --occupancy > gpurun_out/diag.json 2> gpurun_out/err.log
