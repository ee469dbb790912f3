# round 2 checkpoint: smoke, whole GPU suite, default bench, kernel-trace stats of the bench,
# predicted 2/4/8-rank frame times (every share rendered on one GPU)
set -o pipefail
O=gpurun_out/r02chk
mkdir -p $O/prof
R=$GRAFT_REPO_ROOT
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof/kt -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/prof/kt.log 2>&1 || exit 1
for N in 2 4 8; do bash tools/gpu_shard.sh $N || exit 1; done
cp -r gpurun_out/shard $O/
