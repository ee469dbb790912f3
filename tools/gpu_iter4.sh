# parity, then tail-compaction A/B at spp 4/16 and one full-config frame
set -o pipefail
mkdir -p gpurun_out
B="python bench.py --steps 1 --no-cpu-baseline --occupancy"
timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/parity.log 2>&1 &&
timeout -k 10 300 $B --spp 4 --warmup 1 > gpurun_out/r6_s4.json 2> gpurun_out/err.log &&
RT_ROUNDS=0 timeout -k 10 300 $B --spp 4 --warmup 1 > gpurun_out/r0_s4.json 2>> gpurun_out/err.log &&
timeout -k 10 300 $B --spp 16 --warmup 0 > gpurun_out/r6_s16.json 2>> gpurun_out/err.log &&
RT_CHUNKS=1 timeout -k 10 300 $B --spp 16 --warmup 0 > gpurun_out/r6c1_s16.json 2>> gpurun_out/err.log &&
RT_ROUNDS=0 timeout -k 10 300 $B --spp 16 --warmup 0 > gpurun_out/r0_s16.json 2>> gpurun_out/err.log &&
timeout -k 10 400 $B --warmup 0 > gpurun_out/r6_s100.json 2>> gpurun_out/err.log
