set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/latency_probe.py > gpurun_out/lat.json 2> gpurun_out/err.log || exit 1
timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/sp.json 2>> gpurun_out/err.log || exit 1
