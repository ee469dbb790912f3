# INW parity + exactness on one library variant (LIB suffix), then the C3 A/B against the default
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r7; rm -rf $O; mkdir -p $O
V=${V:-_qn}
for L in "" $V; do
  RT_HIP_LIB=$GRAFT_REPO_ROOT/raytracing-tests_amd/librt_hip$L.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bvh_exact.py -k inw -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests$L.log 2>&1 || exit 1
done
NOPARITY=1 bash tools/gpu/ab.sh c3 "- $V" > $O/ab.txt 2>&1 || exit 1
timeout -k 10 200 python3 tools/bench_configs.py --row c5 --spp 64 --reps 3 > $O/c5.jsonl 2> $O/c5.err || exit 1
RT_HIP_LIB=$GRAFT_REPO_ROOT/raytracing-tests_amd/librt_hip$V.so timeout -k 10 200 python3 tools/bench_configs.py --row c5 --spp 64 --reps 3 > $O/c5$V.jsonl 2> $O/c5$V.err || exit 1
