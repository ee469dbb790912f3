# env grid on north-star shares: bash tools/gpu_grid_ns.sh OUT "shares" "ENV.." ...
set -o pipefail
out=$1; shift
shares=$1; shift
mkdir -p gpurun_out/grid
A="--width 1920 --height 1080 --spp 500 --steps 1 --warmup 1 --no-cpu-baseline"
for envs in "$@"; do
  for sh in $shares; do
    f=gpurun_out/grid/$(echo "$out $sh $envs" | tr ' /=' '___').json
    env $envs RT_BENCH_SHARD=$sh timeout -k 10 300 python bench.py $A > $f 2> $f.err || exit 1
    python3 -c "import json;d=json.load(open('$f'));print('$sh', '$envs', d['ms_per_step'], flush=True)" | tee -a gpurun_out/grid/$out.txt
  done
done
