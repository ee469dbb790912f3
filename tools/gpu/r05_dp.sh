# SAH-cost (DP) collapse of the binary SAH tree into 4-wide nodes (RT_COLLAPSE_DP variant) against
# the greedy largest-area collapse: exactness suites on the variant, C3 and C2 A/B
#   gpurun -- 'bash tools/gpu/r05_dp.sh'
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_dp; rm -rf $O; mkdir -p $O
RT_HIP_LIB=raytracing-tests_amd/librt_hip_dp.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_bvh_exact.py > $O/tests.log 2>&1 || exit 1
STEPS=4 bash tools/gpu/r05_ab_variant.sh dp c3 || exit 1
STEPS=1 bash tools/gpu/r05_ab_variant.sh dp c2 || exit 1
echo done
