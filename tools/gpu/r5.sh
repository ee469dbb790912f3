# INW parity + exactness on the default build, A/B of leaf-batch variants, phase split (C3)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_bvh_exact.py -k inw -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/exact_inw.log 2>&1 || exit 1
NOPARITY= bash tools/gpu/ab.sh c3 "${VARS:-- _lb8 _lb24}" > $O/ab.txt 2>&1 || exit 1
RT_HIP_LIB=$GRAFT_REPO_ROOT/raytracing-tests_amd/librt_hip_split.so timeout -k 10 200 python3 tools/inw_split.py c3 500 > $O/split_c3.json 2> $O/split.err || exit 1
