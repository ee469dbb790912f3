# north-star workload: 1 GPU and the 8 shares, default vs 12 checkpoint rounds (same box)
set -o pipefail
O=gpurun_out/nsk
rm -rf $O && mkdir -p $O
A="--width 1920 --height 1080 --spp 500 --steps 1 --warmup 1 --no-cpu-baseline"
for k in 24 12; do
  RT_SPEC_ROUNDS=$k timeout -k 10 300 python3 -u bench.py $A > $O/n1_$k.json 2>> $O/err.log || exit 1
  for r in 0 1 2 3 4 5 6 7; do
    RT_SPEC_ROUNDS=$k RT_BENCH_SHARD=$r/8 timeout -k 10 200 python3 -u bench.py $A > $O/b8_${k}_$r.json 2>> $O/err.log || exit 1
  done
done
python3 - <<'PY'
import json
for k in (24, 12):
    n1 = json.load(open(f"gpurun_out/nsk/n1_{k}.json"))["ms_per_step"]
    t = [json.load(open(f"gpurun_out/nsk/b8_{k}_{r}.json"))["ms_per_step"] for r in range(8)]
    print(k, "1 GPU", round(n1), "8-way max", round(max(t)), "speedup", round(n1 / max(t), 2), [round(x) for x in t])
PY
