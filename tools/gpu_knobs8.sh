# scheduler knobs on the slowest 8-way shares of the bench frame (each share rendered alone)
set -o pipefail
O=gpurun_out/knobs8
rm -rf $O && mkdir -p $O
run() {  # name, env...
  local name=$1; shift
  for r in 2 0 3; do
    env "$@" RT_BENCH_SHARD=$r/8 timeout -k 10 120 python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/${name}_$r.json 2>> $O/err.log || exit 1
  done
}
run A RT_SPEC_TAIL_BUDGET=3072 || exit 1
run B RT_SPEC_TAIL_BUDGET=6144 RT_SPEC_TAIL_ROUNDS=30 || exit 1
run C RT_SPEC_TAIL_BUDGET=1536 RT_SPEC_TAIL_ROUNDS=90 || exit 1
run D RT_SPEC_ROUNDS=12 || exit 1
run E RT_SPEC_ROUNDS=40 || exit 1
run F RT_SPEC_TAIL_ROUNDS=90 || exit 1
python3 - <<'PY'
import json, glob
for n in "ABCDEF":
    t = [json.load(open(f"gpurun_out/knobs8/{n}_{r}.json"))["ms_per_step"] for r in (2, 0, 3)]
    print(n, round(max(t)), [round(x) for x in t])
PY
