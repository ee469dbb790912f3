set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 300 python tools/ab_exact.py 300 200 8 - RT_IOW_NARROW=1 > gpurun_out/ab/ab2.txt 2>&1 || exit 1
for v in 1 0; do
  RT_IOW_LDS=$v timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/ab/bench_$v.json 2> gpurun_out/ab/bench_$v.err || exit 1
done
timeout -k 10 300 python tools/latency_probe.py > gpurun_out/ab/lat.json 2> gpurun_out/ab/lat.err || exit 1
