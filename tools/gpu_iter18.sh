# prior guess + one re-run pass + validated sequential leftovers: neighbours of the best point
set -o pipefail
mkdir -p gpurun_out/v18
B="python bench.py --steps 1 --warmup 0 --no-cpu-baseline"
for cfg in "1 1" "2 0" "2 1" "3 1" "2 1 fix"; do
  set -- $cfg
  F=0; [ "$3" = fix ] && F=1
  RT_SPEC_PRIOR_FROM=$1 RT_SPEC_ITERS=$2 RT_SPEC_FIX=$F timeout -k 10 300 $B > gpurun_out/v18/pf$1_it$2_f$F.json 2>> gpurun_out/v18/err.log || exit 1
done
RT_SPEC_PRIOR_FROM=2 RT_SPEC_ITERS=1 timeout -k 10 300 $B --occupancy > gpurun_out/v18/occ.json 2>> gpurun_out/v18/err.log || exit 1
