# 8-way shares of the bench frame, default build vs the id-dirs reuse variant; INW parity tests
set -o pipefail
O=gpurun_out/var7
rm -rf $O && mkdir -p $O
L=raytracing-tests_amd
for v in "" _idd; do
  for r in 0 1 2 3 4 5 6 7; do
    RT_HIP_LIB=$L/librt_hip$v.so RT_BENCH_COSTS=$O/costs8$v.npy RT_BENCH_SHARD=$r/8 timeout -k 10 200 python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/b8${v}_$r.json 2>> $O/b8.err || exit 1
  done
done
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py > $O/tests.log 2>&1 || exit 1
