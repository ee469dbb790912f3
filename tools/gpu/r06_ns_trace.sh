# Kernel traces of the north-star frame and of its 8-way share 3/8: per-launch durations show
# which phases of the speculation do not shrink with the share (profiles/r06_ns_share_trace.json).
#   gpurun -- 'bash tools/gpu/r06_ns_trace.sh'
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_ns_trace; rm -rf $O; mkdir -p $O
A="--config ns --steps 1 --warmup 1 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/n1 -o run --output-format csv -- python3 bench.py $A > $O/n1.json 2> $O/n1.err || exit 1
RT_BENCH_SHARD=3/8 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/s3 -o run --output-format csv -- python3 bench.py $A > $O/s3.json 2> $O/s3.err || exit 1
echo done
