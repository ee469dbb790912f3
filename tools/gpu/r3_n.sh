# C3 A/B against the pre-prefetch library (same box), the INW tail timeline (full frame and
# 8-way shares), and the north-star slowest share's long-sample timeline
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd "$R"
O=gpurun_out/r3n
rm -rf $O && mkdir -p $O
L=$R/raytracing-tests_amd
run() { timeout -k 10 300 python3 tools/bench_configs.py "$@" >> $O/rows.jsonl 2>> $O/rows.err; }
for i in 1 2; do
  RT_HIP_LIB=$L/librt_hip_old.so run --row c3 --spp 500 --reps 2 || exit 1
  run --row c3 --spp 500 --reps 2 || exit 1
done
S="timeout -k 10 200 env RT_HIP_LIB=$L/librt_hip_split.so python3 tools/inw_split.py"
$S c3 500 > $O/split_full.json 2>> $O/split.err || exit 1
$S c3 500 6/8 > $O/split_s6.json 2>> $O/split.err || exit 1
$S c3 500 1/8 > $O/split_s1.json 2>> $O/split.err || exit 1
RT_HIP_LIB=$L/librt_hip_diag.so timeout -k 10 300 python3 tools/spec_times.py 6 8 > $O/ns_times_s6.json 2> $O/ns_times.err || exit 1
timeout -k 10 300 python3 bench.py --config c2 --steps 1 --warmup 1 --no-cpu-baseline --occupancy > $O/c2_occ.json 2> $O/c2_occ.err || exit 1
