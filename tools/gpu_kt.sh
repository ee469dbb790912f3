# kernel trace of one bench frame
set -o pipefail
mkdir -p gpurun_out/kt
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/kt/kt.log 2>&1 || exit 1
