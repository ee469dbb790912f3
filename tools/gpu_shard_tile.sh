# 8-way shard times for other tile sizes: bash tools/gpu_shard_tile.sh 16 32
set -o pipefail
mkdir -p gpurun_out/shtile
for T in "$@"; do
  for r in 0 1 2 3 4 5 6 7; do
    RT_BENCH_TILE=$T RT_BENCH_SHARD=$r/8 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/shtile/t${T}_$r.json 2> gpurun_out/shtile/t${T}_$r.err || exit 1
  done
  python3 -c "
import json
t=[json.load(open('gpurun_out/shtile/t${T}_%d.json'%r))['ms_per_step'] for r in range(8)]
print('tile $T max', max(t), t)"
done
