set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --spp 4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/b_spp4.json 2> gpurun_out/b_spp4.err
timeout -k 10 600 python bench.py --spp 16 --steps 1 --warmup 0 --cpu-px 8 > gpurun_out/b_spp16.json 2> gpurun_out/b_spp16.err
