# Sphere-record hit normals, built as librt_hip_sphn.so, against the same source with
# -DRT_INW_SPH_NO_NORMAL (librt_hip_nonorm.so): exactness suites on the variant, then C3 A/B.
#   gpurun -- 'bash tools/gpu/r06_sphn.sh'
set -o pipefail
O=gpurun_out/r06_sphn; rm -rf $O; mkdir -p $O
L=$GRAFT_REPO_ROOT/raytracing-tests_amd
RT_HIP_LIB=$L/librt_hip_sphn.so timeout -k 10 1000 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_bvh_exact.py tests/test_gpu_parity.py tests/test_gpu_fullspp.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  RT_HIP_LIB=$L/librt_hip_sphn.so timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 > $O/c3n_$i.json 2> $O/c3n_$i.err || exit 1
  RT_HIP_LIB=$L/librt_hip_nonorm.so timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 > $O/c3old_$i.json 2> $O/c3old_$i.err || exit 1
done
echo done
