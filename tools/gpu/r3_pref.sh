# fold-window prefetch in k_inw_pm: parity, exactness, C3 timing and phase split
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd "$R"
O=gpurun_out/r3l
rm -rf $O && mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "inw or tile_list" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/parity.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_bvh_exact.py -k "inw" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/exact_inw.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/bench_configs.py --row c3 --spp 500 --reps 2 >> $O/rows.jsonl 2>> $O/rows.err || exit 1
RT_HIP_LIB=$R/raytracing-tests_amd/librt_hip_split.so timeout -k 10 200 python3 tools/inw_split.py c3 > $O/split_c3.json 2>&1 || exit 1
