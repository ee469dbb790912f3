set -o pipefail
mkdir -p gpurun_out/tail
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python tools/ab_exact.py 300 200 16 RT_SPEC_TAIL_ROUNDS=0 - RT_SPEC_TAIL_BUDGET=64,RT_SPEC_TAIL_ROUNDS=30 > gpurun_out/tail/ab.txt 2>&1 || exit 1
for v in "RT_SPEC_HEAVY=5" "RT_SPEC_HEAVY=5,RT_SPEC_TAIL_BUDGET=16384,RT_SPEC_TAIL_ROUNDS=16" "RT_SPEC_HEAVY=5,RT_SPEC_TAIL_BUDGET=2048,RT_SPEC_TAIL_ROUNDS=100"; do
  env $(echo $v | tr ',' ' ') timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/tail/bench_$v.json 2> gpurun_out/tail/bench_$v.err || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd "$R"
RT_SPEC_HEAVY=5 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tail/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/tail/kt.log 2>&1 || exit 1
