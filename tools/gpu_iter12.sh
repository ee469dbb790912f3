set -o pipefail
mkdir -p gpurun_out
B="python bench.py --steps 1 --warmup 0 --no-cpu-baseline"
for t in 1000000 4 16 40; do
  RT_SPEC_PRIOR_FROM=$t timeout -k 10 300 $B > gpurun_out/pf_$t.json 2>> gpurun_out/err.log || exit 1
done
