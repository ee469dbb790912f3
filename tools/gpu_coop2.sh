# coop v2: lone-lane probe, exactness, bench sweep
set -o pipefail
mkdir -p gpurun_out/probe2
timeout -k 10 300 python tools/latency_probe.py > gpurun_out/probe2/lat.json 2> gpurun_out/probe2/lat.err || exit 1
timeout -k 10 500 python -u -m pytest tests/test_gpu_bvh_exact.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/probe2/exact.log 2>&1 || exit 1
for c in 0 4 8 16; do
  RT_COOP=$c timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/probe2/bench_$c.json 2> gpurun_out/probe2/bench_$c.err || exit 1
done
