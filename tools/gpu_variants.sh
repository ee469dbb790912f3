# A/B of scheduler switches on one rank's share of an N-way partition: bash tools/gpu_variants.sh R N "VAR=a,VAR2=b" ...
# (R/N = 0/1 is the whole bench frame)
set -o pipefail
r=$1; n=$2; shift 2
mkdir -p gpurun_out/var
i=0
for v in "$@"; do
  i=$((i+1))
  env $(echo $v | tr ',' ' ') RT_BENCH_SHARD=$r/$n timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/var/b_${r}_${n}_$i.json 2> gpurun_out/var/b_${r}_${n}_$i.err || exit 1
  echo "$v $(python -c "import json;d=json.load(open('gpurun_out/var/b_${r}_${n}_$i.json'));print(d['ms_per_step'], d['rays_per_step'])")"
done
