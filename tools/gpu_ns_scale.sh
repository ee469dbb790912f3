# north-star workload (IOW-03 final scene, 1920x1080, 500 spp, 50 bounces): 1 GPU and every
# share of an 8-way tile partition rendered alone on one GPU (predicted 8-GPU frame = max)
set -o pipefail
O=gpurun_out/ns
mkdir -p $O
A="--width 1920 --height 1080 --spp 500 --steps 1 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 python bench.py $A > $O/n1.json 2> $O/n1.err || exit 1
for r in 0 1 2 3 4 5 6 7; do
  RT_BENCH_COSTS=$O/costs_ns8.npy RT_BENCH_SHARD=$r/8 timeout -k 10 200 python bench.py $A > $O/b8_$r.json 2> $O/b8_$r.err || exit 1
done
python3 - <<'PY'
import json
n1 = json.load(open("gpurun_out/ns/n1.json"))["ms_per_step"]
t = [json.load(open(f"gpurun_out/ns/b8_{r}.json"))["ms_per_step"] for r in range(8)]
print("1 GPU", n1, "8-way max", max(t), "speedup", round(n1 / max(t), 2), [round(x) for x in t])
PY
