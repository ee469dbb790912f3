# LDS-staged BVH: smoke, full GPU suite, bench A/B
set -o pipefail
mkdir -p gpurun_out/lds
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/lds/smoke.log 2>&1 || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/lds/gpu_tests.log 2>&1 || exit 1
for v in 1 0; do
  RT_IOW_LDS=$v timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/lds/bench_$v.json 2> gpurun_out/lds/bench_$v.err || exit 1
done
timeout -k 10 300 python tools/latency_probe.py > gpurun_out/lds/lat.json 2> gpurun_out/lds/lat.err || exit 1
