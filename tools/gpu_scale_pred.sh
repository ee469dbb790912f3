# predicted strong-scaling curve: every rank's share of 2-, 4- and 8-way tile partitions,
# rendered one share at a time on one GPU (the N-GPU frame time is the max over ranks)
set -o pipefail
mkdir -p gpurun_out/shard
for N in 2 4 8; do
  bash tools/gpu_shard.sh $N || exit 1
done
python3 - <<'PY'
import json
for N in (2, 4, 8):
    t = [json.load(open(f"gpurun_out/shard/b{N}_{r}.json"))["ms_per_step"] for r in range(N)]
    print(N, "max_ms", max(t), "per_rank_ms", t)
PY
