set -o pipefail
mkdir -p gpurun_out/ckpt2
R=$GRAFT_REPO_ROOT
for k in 24 32 40; do
  RT_SPEC_ROUNDS=$k timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/ckpt2/bench_$k.json 2> gpurun_out/ckpt2/bench_$k.err || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd "$R"
RT_SPEC_ROUNDS=32 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ckpt2/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/ckpt2/kt.log 2>&1 || exit 1
