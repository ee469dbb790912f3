set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -s -p no:cacheprovider > gpurun_out/parity.log 2>&1
timeout -k 10 600 python bench.py --spp 4 --steps 1 --warmup 1 --no-cpu-baseline --occupancy > gpurun_out/occ.json 2> gpurun_out/occ.err
timeout -k 10 600 python bench.py --spp 16 --steps 1 --warmup 0 --no-cpu-baseline --occupancy > gpurun_out/occ16.json 2> gpurun_out/occ16.err
