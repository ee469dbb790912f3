# re-entry check: smoke, full GPU suite, default bench line, kernel trace of one frame
set -o pipefail
mkdir -p gpurun_out/r1b/prof
R=$GRAFT_REPO_ROOT
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r1b/smoke.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r1b/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/r1b/bench_default.json 2> gpurun_out/r1b/bench_default.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r1b/prof/kt -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r1b/prof/kt.log 2>&1 || exit 1
