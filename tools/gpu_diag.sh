set -o pipefail
mkdir -p gpurun_out/diag
for c in 0 4; do
RT_COOP=$c timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --occupancy > gpurun_out/diag/diag_$c.json 2> gpurun_out/diag/err_$c.log || exit 1
done
