# env grid over bench.py shares: bash tools/gpu_grid.sh OUT "share ..." "ENV=.. ENV=.." ...
# prints share, env, ms_per_step per run (one bench frame after a warm-up frame)
set -o pipefail
out=$1; shift
shares=$1; shift
mkdir -p gpurun_out/grid
for envs in "$@"; do
  for sh in $shares; do
    f=gpurun_out/grid/$(echo "$out $sh $envs" | tr ' /=' '___').json
    env $envs RT_BENCH_SHARD=$sh timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > $f 2> $f.err || exit 1
    python3 -c "import json;d=json.load(open('$f'));print('$sh', '$envs', d['ms_per_step'], d['value'], flush=True)" | tee -a gpurun_out/grid/$out.txt
  done
done
