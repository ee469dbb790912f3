# Unrotated-object fast path in the wide walk object test (default) against -DRT_INW_NO_IDENT
# (librt_hip_noid.so): exactness suites, then C5 and C3 A/B.
#   gpurun -- 'bash tools/gpu/r06_ident.sh'
set -o pipefail
O=gpurun_out/r06_ident; rm -rf $O; mkdir -p $O
V=$GRAFT_REPO_ROOT/raytracing-tests_amd/librt_hip_noid.so
timeout -k 10 1000 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_bvh_exact.py tests/test_gpu_parity.py tests/test_gpu_fullspp.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 bench.py --config c5 --no-cpu-baseline --steps 1 > $O/c5id_1.json 2> $O/c5id_1.err || exit 1
RT_HIP_LIB=$V timeout -k 10 300 python3 bench.py --config c5 --no-cpu-baseline --steps 1 > $O/c5noid_1.json 2> $O/c5noid_1.err || exit 1
timeout -k 10 300 python3 bench.py --config c5 --no-cpu-baseline --steps 1 > $O/c5id_2.json 2> $O/c5id_2.err || exit 1
RT_HIP_LIB=$V timeout -k 10 300 python3 bench.py --config c5 --no-cpu-baseline --steps 1 > $O/c5noid_2.json 2> $O/c5noid_2.err || exit 1
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 > $O/c3id_1.json 2> $O/c3id_1.err || exit 1
RT_HIP_LIB=$V timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 > $O/c3noid_1.json 2> $O/c3noid_1.err || exit 1
echo done
