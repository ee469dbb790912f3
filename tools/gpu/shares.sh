# Predicted strong scaling: every rank's share of an N-way tile partition rendered alone on one
# GPU (the N-GPU frame time is the max over ranks), against the 1-GPU frame.
#   gpurun -- 'bash tools/gpu/shares.sh c3 8 [steps] [bench args, e.g. --opt spec_heavy=48]'
set -o pipefail
CFG=${1:-c3}; N=${2:-8}; K=${3:-1}
shift 3 2>/dev/null || shift $#
O=gpurun_out/shares_${CFG}_$N
rm -rf $O && mkdir -p $O
A="--config $CFG --steps $K --warmup 1 --no-cpu-baseline $*"
timeout -k 10 600 python3 bench.py $A > $O/n1.json 2> $O/n1.err || exit 1
for r in $(seq 0 $((N - 1))); do
  RT_BENCH_SHARD=$r/$N timeout -k 10 300 python3 bench.py $A > $O/s$r.json 2> $O/s$r.err || exit 1
done
python3 - "$O" "$N" > $O/summary.json <<'PY' || exit 1
import json, sys
o, n = sys.argv[1], int(sys.argv[2])
one = json.load(open(f"{o}/n1.json"))
sh = [json.load(open(f"{o}/s{r}.json")) for r in range(n)]
t = [s["ms_per_step"] for s in sh]
kt = [s["roofline"]["main_kernel_ms_per_frame"] for s in sh]
print(json.dumps({"config": one["config"]["workload"], "n1_ms": one["ms_per_step"],
                  "n1_kernel_ms": one["roofline"]["main_kernel_ms_per_frame"], "ranks": n,
                  "share_ms": t, "share_kernel_ms": kt, "max_share_ms": max(t),
                  "predicted_speedup": round(one["ms_per_step"] / max(t), 3)}))
PY
cat $O/summary.json
