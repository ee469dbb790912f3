# LDS coop cull: lone-pixel split (diag build), parity tests, bench frame x2
set -o pipefail
O=gpurun_out/var4
rm -rf $O && mkdir -p $O
L=raytracing-tests_amd
RT_HIP_LIB=$L/librt_hip_diag.so timeout -k 10 200 python3 -u tools/variant_probe.py > $O/probe_diag.json 2> $O/probe_diag.err || exit 1
for i in 1 2; do
  timeout -k 10 200 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline >> $O/bench.jsonl 2>> $O/bench.err || exit 1
done
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bvh_exact.py tests/test_gpu_parity.py > $O/tests.log 2>&1 || exit 1
