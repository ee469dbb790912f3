# per-rank frame time of an N-way tile partition (N = $1, default 8), rendered shard by shard
# on one GPU: predicts the N-GPU frame time (max over ranks) before the driver's scaling run
set -o pipefail
N=${1:-8}
mkdir -p gpurun_out/shard
for r in $(seq 0 $((N-1))); do
  RT_BENCH_SHARD=$r/$N timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/shard/b${N}_$r.json 2> gpurun_out/shard/b${N}_$r.err || exit 1
done
