# tail analysis: per-pixel ray distribution, per-round parked lanes, park_min / rounds variants
set -o pipefail
mkdir -p gpurun_out
B="python bench.py --steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 300 $B --occupancy > gpurun_out/t_occ.json 2> gpurun_out/err.log || exit 1
RT_PARK_MIN=0 RT_ROUNDS=14 timeout -k 10 300 $B --occupancy > gpurun_out/t_occ_p0.json 2>> gpurun_out/err.log || exit 1
RT_PARK_MIN=0 RT_ROUNDS=14 timeout -k 10 300 $B > gpurun_out/t_p0.json 2>> gpurun_out/err.log || exit 1
