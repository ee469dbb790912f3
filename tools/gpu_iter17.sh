# record validation in the sequential fallback: exactness tests, then a guess x iterations grid
set -o pipefail
mkdir -p gpurun_out/v17
timeout -k 10 900 python -m pytest tests/test_gpu_bvh_exact.py -q -x -p no:cacheprovider > gpurun_out/v17/exact.log 2>&1 || exit 1
B="python bench.py --steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 300 $B > gpurun_out/v17/def.json 2>> gpurun_out/v17/err.log || exit 1
RT_SPEC_VALIDATE=0 timeout -k 10 300 $B > gpurun_out/v17/noval.json 2>> gpurun_out/v17/err.log || exit 1
for pf in 20 8 2; do for it in 1 2 4; do
  RT_SPEC_PRIOR_FROM=$pf RT_SPEC_ITERS=$it timeout -k 10 300 $B > gpurun_out/v17/pf${pf}_it${it}.json 2>> gpurun_out/v17/err.log || exit 1
done; done
for it in 1 2 4; do
  RT_SPEC_ITERS=$it timeout -k 10 300 $B > gpurun_out/v17/it${it}.json 2>> gpurun_out/v17/err.log || exit 1
done
