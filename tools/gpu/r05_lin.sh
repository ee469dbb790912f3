# Few-object linear closest hit (RT_INW_LINEAR_MAX variant): exactness suites on the variant, then
# the C5 A/B against the product library
#   gpurun -- 'bash tools/gpu/r05_lin.sh'
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_lin; rm -rf $O; mkdir -p $O
RT_HIP_LIB=raytracing-tests_amd/librt_hip_lin.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_bvh_exact.py tests/test_gpu_textures.py > $O/tests.log 2>&1 || exit 1
STEPS=2 bash tools/gpu/r05_ab_variant.sh lin c5 || exit 1
echo done
