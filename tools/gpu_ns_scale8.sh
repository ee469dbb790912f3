# 8-way shares only (the 1-GPU frame from an earlier run): north-star workload and the bench frame
set -o pipefail
O=gpurun_out/ns2
mkdir -p $O
A="--width 1920 --height 1080 --spp 500 --steps 1 --warmup 1 --no-cpu-baseline"
for r in 0 1 2 3 4 5 6 7; do
  RT_BENCH_SHARD=$r/8 timeout -k 10 200 python bench.py $A > $O/b8_$r.json 2> $O/b8_$r.err || exit 1
done
bash tools/gpu_shard.sh 8 || exit 1
python3 - <<'PY'
import json
t = [json.load(open(f"gpurun_out/ns2/b8_{r}.json"))["ms_per_step"] for r in range(8)]
print("north-star 8-way max", max(t), [round(x) for x in t])
t = [json.load(open(f"gpurun_out/shard/b8_{r}.json"))["ms_per_step"] for r in range(8)]
print("C2 8-way max", max(t), [round(x) for x in t])
PY
