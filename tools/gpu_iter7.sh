# parity, then leaf-batch sweep at the full config
set -o pipefail
mkdir -p gpurun_out
B="python bench.py --steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/parity.log 2>&1 || exit 1
for b in 65 48 32; do
  RT_LEAF_BATCH=$b timeout -k 10 300 $B > gpurun_out/lb_$b.json 2>> gpurun_out/err.log || exit 1
done
timeout -k 10 300 $B --occupancy > gpurun_out/lb_occ.json 2>> gpurun_out/err.log
