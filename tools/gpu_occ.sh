set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --spp 4 --steps 1 --warmup 0 --no-cpu-baseline --occupancy > gpurun_out/occ.json 2> gpurun_out/occ.err
