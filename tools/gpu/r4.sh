set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r4; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bvh_exact.py -k inw -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests_inw.log 2>&1 || exit 1
RT_INW_FAST=0 timeout -k 10 200 python3 bench.py --config c3 --steps 1 --warmup 0 --no-cpu-baseline > $O/c3_refwalk.json 2> $O/c3_refwalk.err || exit 1
RT_HIP_LIB=$GRAFT_REPO_ROOT/raytracing-tests_amd/librt_hip_split.so timeout -k 10 200 python3 tools/inw_split.py c3 500 > $O/split_c3.json 2> $O/split.err || exit 1
for v in "" _base; do
  RT_HIP_LIB=$GRAFT_REPO_ROOT/raytracing-tests_amd/librt_hip$v.so timeout -k 10 200 python3 tools/bench_configs.py --row c5 --spp 64 --reps 3 > $O/c5$v.jsonl 2> $O/c5$v.err || exit 1
  RT_HIP_LIB=$GRAFT_REPO_ROOT/raytracing-tests_amd/librt_hip$v.so timeout -k 10 200 python3 bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/c3$v.json 2> $O/c3$v.err || exit 1
done
RT_INW_LDS=0 timeout -k 10 200 python3 bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/c3_lds0.json 2> $O/c3_lds0.err || exit 1
