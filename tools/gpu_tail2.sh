set -o pipefail
mkdir -p gpurun_out/tail2
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python tools/ab_exact.py 300 200 16 RT_SPEC_SPREAD=0 - RT_SPEC_TAIL_ROUNDS=20 > gpurun_out/tail2/ab.txt 2>&1 || exit 1
for v in "RT_SPEC_SPREAD=0" "RT_SPEC_SPREAD=1" "RT_SPEC_HEAVY=9" "RT_SPEC_TAIL_ROUNDS=8,RT_SPEC_TAIL_BUDGET=16384"; do
  env $(echo $v | tr ',' ' ') timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/tail2/bench_$v.json 2> gpurun_out/tail2/bench_$v.err || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tail2/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/tail2/kt.log 2>&1 || exit 1
