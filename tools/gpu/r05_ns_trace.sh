# Kernel trace of one 8-way share of the north-star frame (IOW-03 1080p, 500 spp): per-launch durations
#   gpurun -- 'bash tools/gpu/r05_ns_trace.sh'
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_ns_trace; rm -rf $O; mkdir -p $O
RT_BENCH_SHARD=0/8 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/kt -o run --output-format csv -- python3 bench.py --config ns --steps 1 --warmup 1 --no-cpu-baseline > $O/share0.json 2> $O/share0.err || exit 1
echo done
