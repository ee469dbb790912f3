set -o pipefail
mkdir -p gpurun_out/heavy
timeout -k 10 400 python tools/ab_exact.py 300 200 16 RT_SPEC_HEAVY=0 - RT_SPEC_HEAVY=3,RT_SPEC_PROBE=7 RT_SPEC_ROUNDS=0 > gpurun_out/heavy/ab.txt 2>&1 || exit 1
for v in "RT_SPEC_HEAVY=0" "RT_SPEC_HEAVY=9" "RT_SPEC_HEAVY=5" "RT_SPEC_HEAVY=20" "RT_SPEC_HEAVY=9,RT_SPEC_ROUNDS=40"; do
  env $(echo $v | tr ',' ' ') timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/heavy/bench_$v.json 2> gpurun_out/heavy/bench_$v.err || exit 1
done
RT_SPEC_HEAVY=9 timeout -k 10 300 python tools/spec_stats.py > gpurun_out/heavy/stats.json 2> gpurun_out/heavy/stats.err || exit 1
