# Predicted strong scaling with the time-refined deal (bench.refine_deal): the hashed deal's shares
# rendered alone (tools/gpu/shares.sh), the per-tile rays of a full frame (RT_BENCH_COSTS), the
# refined lists from those times and rays, then every refined share rendered alone.
#   gpurun -- 'bash tools/gpu/shares_refined.sh ns 8 1 --opt spec_heavy=48'
set -o pipefail
CFG=${1:-c3}; N=${2:-8}; K=${3:-1}
shift 3 2>/dev/null || shift $#
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu/shares.sh $CFG $N $K "$@" > /dev/null || exit 1
O=gpurun_out/shares_${CFG}_$N
R=gpurun_out/refined_${CFG}_$N
rm -rf $R && mkdir -p $R
A="--config $CFG --steps $K --warmup 1 --no-cpu-baseline $*"
# per-tile rays: a shard process with --balance renders every tile in its warm-up and caches them
RT_BENCH_SHARD=0/$N RT_BENCH_COSTS=$R/costs.npy timeout -k 10 600 python3 bench.py $A --balance > $R/costs.json 2> $R/costs.err || exit 1
python3 - "$O" "$R" "$N" "$CFG" <<'PY' || exit 1
import json, math, sys
import numpy as np
sys.path.insert(0, ".")
import bench
o, r, n, cfg = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
one = json.load(open(f"{o}/n1.json"))
W, H = one["config"]["width"], one["config"]["height"]
T = bench.tile_for(n)
nx, ny = math.ceil(W / T), math.ceil(H / T)
order = bench.deal_order(nx, ny, n)
lists = [order[k::n] for k in range(n)]
times = [json.load(open(f"{o}/s{k}.json"))["ms_per_step"] for k in range(n)]
new = bench.refine_deal(lists, np.load(f"{r}/costs.npy"), times, nx)
json.dump([[list(t) for t in lst] for lst in new], open(f"{r}/deal.json", "w"))
print("tiles per rank", [len(l) for l in new])
PY
for k in $(seq 0 $((N - 1))); do
  RT_BENCH_SHARD=$k/$N RT_BENCH_DEAL=$R/deal.json timeout -k 10 300 python3 bench.py $A > $R/s$k.json 2> $R/s$k.err || exit 1
done
python3 - "$O" "$R" "$N" > $R/summary.json <<'PY' || exit 1
import json, sys
o, r, n = sys.argv[1], sys.argv[2], int(sys.argv[3])
one = json.load(open(f"{o}/n1.json"))
h = [json.load(open(f"{o}/s{k}.json"))["ms_per_step"] for k in range(n)]
t = [json.load(open(f"{r}/s{k}.json"))["ms_per_step"] for k in range(n)]
print(json.dumps({"config": one["config"]["workload"], "n1_ms": one["ms_per_step"], "ranks": n,
                  "hashed_share_ms": h, "hashed_speedup": round(one["ms_per_step"] / max(h), 3),
                  "refined_share_ms": t, "refined_speedup": round(one["ms_per_step"] / max(t), 3)}))
PY
cat $R/summary.json
