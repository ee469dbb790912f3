# fused cull as a kernel variant: parity / exactness / C3 timing (A/B vs the pre-prefetch
# library, same box); INW share tails with the share's tiles in deal vs row order
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd "$R"
O=gpurun_out/r3o
rm -rf $O && mkdir -p $O
L=$R/raytracing-tests_amd
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "inw or tile_list" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/parity.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_bvh_exact.py -k "inw" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/exact_inw.log 2>&1 || exit 1
run() { timeout -k 10 300 python3 tools/bench_configs.py "$@" >> $O/rows.jsonl 2>> $O/rows.err; }
for i in 1 2; do
  RT_HIP_LIB=$L/librt_hip_old.so run --row c3 --spp 500 --reps 2 || exit 1
  run --row c3 --spp 500 --reps 2 || exit 1
done
RT_INW_FMA=0 run --row c3 --spp 500 --reps 2 || exit 1
run --row c5 --spp 64 --reps 2 || exit 1
S="timeout -k 10 200 env RT_HIP_LIB=$L/librt_hip_split.so python3 tools/inw_split.py"
for r in 1 6; do
  $S c3 500 $r/8 > $O/split_s$r.json 2>> $O/split.err || exit 1
  RT_SPLIT_ROWS=1 $S c3 500 $r/8 > $O/split_rows_s$r.json 2>> $O/split.err || exit 1
done
