# cost-ordered claims (RT_INW_COST): parity / exactness, C3 + C5 timing on/off, share tails
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd "$R"
O=gpurun_out/r3p
rm -rf $O && mkdir -p $O
L=$R/raytracing-tests_amd
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "inw or tile_list" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/parity.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_bvh_exact.py -k "inw" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/exact_inw.log 2>&1 || exit 1
run() { timeout -k 10 300 python3 tools/bench_configs.py "$@" >> $O/rows.jsonl 2>> $O/rows.err; }
run --row c3 --spp 500 --reps 2 || exit 1
RT_INW_COST=0 run --row c3 --spp 500 --reps 2 || exit 1
run --row c5 --spp 64 --reps 2 || exit 1
RT_INW_COST=0 run --row c5 --spp 64 --reps 2 || exit 1
S="timeout -k 10 200 env RT_HIP_LIB=$L/librt_hip_split.so python3 tools/inw_split.py"
$S c3 500 > $O/split_full.json 2>> $O/split.err || exit 1
for r in 1 6; do
  $S c3 500 $r/8 > $O/split_s$r.json 2>> $O/split.err || exit 1
done
bash tools/gpu/shares.sh c3 8 3 > $O/shares.log 2>&1 || exit 1
