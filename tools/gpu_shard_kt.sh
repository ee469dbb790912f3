# kernel trace of one rank's share of an N-way tile partition (rank $1 of $2), one frame
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/shkt
cd /tmp && export TMPDIR=/tmp && cd "$R"
RT_BENCH_SHARD=$1/$2 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/shkt/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/shkt/kt.log 2>&1 || exit 1
