# checkpoint rounds: exactness A/B, then bench frame for several round counts
set -o pipefail
mkdir -p gpurun_out/ckpt
timeout -k 10 400 python tools/ab_exact.py 300 200 16 - RT_SPEC_ROUNDS=8 RT_SPEC_ROUNDS=24,RT_SPEC_PRIOR_FROM=1 RT_SPEC_ROUNDS=5,RT_SPEC_GROUPS=3 > gpurun_out/ckpt/ab.txt 2>&1 || exit 1
for k in 0 8 16 32; do
  RT_SPEC_ROUNDS=$k timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/ckpt/bench_$k.json 2> gpurun_out/ckpt/bench_$k.err || exit 1
done
