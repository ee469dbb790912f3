# Scalar-load node steps (-DRT_INW_NODE_SLOAD, librt_hip_nsl.so): INW exactness tests on the
# variant, then C3 A/B against the product library.
#   gpurun -- 'bash tools/gpu/r06_nsl.sh'
set -o pipefail
O=gpurun_out/r06_nsl; rm -rf $O; mkdir -p $O
V=$GRAFT_REPO_ROOT/raytracing-tests_amd/librt_hip_nsl.so
RT_HIP_LIB=$V timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bvh_exact.py -k "inw" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 > $O/prod_$i.json 2> $O/prod_$i.err || exit 1
  RT_HIP_LIB=$V timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 > $O/nsl_$i.json 2> $O/nsl_$i.err || exit 1
done
echo done
