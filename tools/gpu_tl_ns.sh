# kernel timeline of one north-star share: bash tools/gpu_tl_ns.sh 3/8
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd "$R"
sh=$1
d=gpurun_out/tlns/$(echo $sh | tr '/' '_')
rm -rf $d && mkdir -p $d
RT_BENCH_SHARD=$sh timeout -k 10 300 rocprofv3 --kernel-trace -d $d/prof -o run --output-format csv -- python3 bench.py --width 1920 --height 1080 --spp 500 --steps 1 --warmup 0 --no-cpu-baseline > $d/kt.log 2>&1 || exit 1
