# kernel timelines (launches > 2 ms) of rank R of N shares: bash tools/gpu/timeline.sh "0/1" "5/8" ...
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd "$R"
for sh in "$@"; do
  d=gpurun_out/tl/$(echo $sh | tr '/' '_')
  rm -rf $d && mkdir -p $d
  RT_BENCH_SHARD=$sh timeout -k 10 300 rocprofv3 --kernel-trace -d $d/prof -o run --output-format csv -- python3 bench.py --config c2 --steps 1 --warmup 0 --no-cpu-baseline > $d/kt.log 2>&1 || exit 1
  echo "== $sh"; python3 tools/timeline.py $(find $d -name "*kernel_trace.csv" | head -1) 2 | tail -20
done
