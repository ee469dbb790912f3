# per-rank frame time of an 8-way tile partition, rendered shard by shard on one GPU
set -o pipefail
mkdir -p gpurun_out/shard
for v in "RT_SPEC_TAIL_ROUNDS=0" "RT_SPEC_TAIL_ROUNDS=20"; do
for r in 0 1 2 3 4 5 6 7; do
  env $(echo $v | tr ',' ' ') RT_BENCH_SHARD=$r/8 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/shard/b_${v}_$r.json 2> gpurun_out/shard/b_${v}_$r.err || exit 1
done
done
