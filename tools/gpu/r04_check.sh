# Round-4 check of the default build: INW + IOW parity and exactness suites, full-spp parity, bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_check; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bvh_exact.py tests/test_gpu_fullspp.py tests/test_gpu_textures.py tests/test_gpu_stages.py -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { echo TESTS_FAILED; exit 1; }
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 1
RT_HIP_LIB=$GRAFT_REPO_ROOT/raytracing-tests_amd/librt_hip_occ.so timeout -k 10 200 python3 tools/inw_occ.py c3 > $O/occ_c3.json 2> $O/occ_c3.err || exit 1
RT_HIP_LIB=$GRAFT_REPO_ROOT/raytracing-tests_amd/librt_hip_occ.so timeout -k 10 200 python3 tools/inw_occ.py c5 64 > $O/occ_c5.json 2> $O/occ_c5.err || exit 1
