# wave-cooperative closest hits: exactness vs the other strategies, then the bench frame at several thresholds
set -o pipefail
mkdir -p gpurun_out/coop
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/coop/smoke.log 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest tests/test_gpu_bvh_exact.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/coop/exact.log 2>&1 || exit 1
for c in 0 4 1 8 16; do
  RT_COOP=$c timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/coop/bench_$c.json 2> gpurun_out/coop/bench_$c.err || exit 1
done
