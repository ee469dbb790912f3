# The refined leaf-entry guard (the best hit's box entry against the other hits' t) against the
# round-5 guard (-DRT_INW_GUARD_ANY, librt_hip_gany.so): exactness suites, then C5 and C3 A/B.
#   gpurun -- 'bash tools/gpu/r06_guard.sh'
set -o pipefail
O=gpurun_out/r06_guard; rm -rf $O; mkdir -p $O
V=$GRAFT_REPO_ROOT/raytracing-tests_amd/librt_hip_gany.so
timeout -k 10 1000 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_bvh_exact.py tests/test_gpu_parity.py tests/test_gpu_fullspp.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 bench.py --config c5 --no-cpu-baseline --steps 1 > $O/c5new_1.json 2> $O/c5new_1.err || exit 1
RT_HIP_LIB=$V timeout -k 10 300 python3 bench.py --config c5 --no-cpu-baseline --steps 1 > $O/c5old_1.json 2> $O/c5old_1.err || exit 1
timeout -k 10 300 python3 bench.py --config c5 --no-cpu-baseline --steps 1 > $O/c5new_2.json 2> $O/c5new_2.err || exit 1
RT_HIP_LIB=$V timeout -k 10 300 python3 bench.py --config c5 --no-cpu-baseline --steps 1 > $O/c5old_2.json 2> $O/c5old_2.err || exit 1
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 > $O/c3new_1.json 2> $O/c3new_1.err || exit 1
RT_HIP_LIB=$V timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 > $O/c3old_1.json 2> $O/c3old_1.err || exit 1
echo done
