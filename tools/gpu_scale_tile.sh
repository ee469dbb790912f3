# every rank's share of 1/2/4-way partitions with tile edge $1 (8-way: tools/gpu_shard_tile.sh)
set -o pipefail
mkdir -p gpurun_out/shtile
T=$1
for N in 1 2 4; do
  for r in $(seq 0 $((N-1))); do
    RT_BENCH_TILE=$T RT_BENCH_SHARD=$r/$N timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/shtile/t${T}_n${N}_$r.json 2> gpurun_out/shtile/t${T}_n${N}_$r.err || exit 1
  done
  python3 -c "
import json
t=[json.load(open('gpurun_out/shtile/t${T}_n${N}_%d.json'%r))['ms_per_step'] for r in range($N)]
print('tile $T N $N max', max(t), t)"
done
