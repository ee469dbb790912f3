# Unrotated-object hit normals (librt_hip_idn.so) against the same source without them
# (librt_hip_base.so): exactness suites on the variant, then C5 and C3 A/B.
#   gpurun -- 'bash tools/gpu/r06_idn.sh'
set -o pipefail
O=gpurun_out/r06_idn; rm -rf $O; mkdir -p $O
L=$GRAFT_REPO_ROOT/raytracing-tests_amd
RT_HIP_LIB=$L/librt_hip_idn.so timeout -k 10 1000 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_bvh_exact.py tests/test_gpu_parity.py tests/test_gpu_fullspp.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  RT_HIP_LIB=$L/librt_hip_idn.so timeout -k 10 300 python3 bench.py --config c5 --no-cpu-baseline --steps 1 > $O/c5n_$i.json 2> $O/c5n_$i.err || exit 1
  RT_HIP_LIB=$L/librt_hip_base.so timeout -k 10 300 python3 bench.py --config c5 --no-cpu-baseline --steps 1 > $O/c5b_$i.json 2> $O/c5b_$i.err || exit 1
done
RT_HIP_LIB=$L/librt_hip_idn.so timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 > $O/c3n_1.json 2> $O/c3n_1.err || exit 1
RT_HIP_LIB=$L/librt_hip_base.so timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 > $O/c3b_1.json 2> $O/c3b_1.err || exit 1
echo done
