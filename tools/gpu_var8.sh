# compiler scheduling strategy max-ilp vs default: bench frame x2 each, INW configs
set -o pipefail
O=gpurun_out/var8
rm -rf $O && mkdir -p $O
L=raytracing-tests_amd
for v in "" _ilp "" _ilp; do
  RT_HIP_LIB=$L/librt_hip$v.so timeout -k 10 200 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline >> $O/bench$v.jsonl 2>> $O/bench.err || exit 1
done
for v in "" _ilp; do
  RT_HIP_LIB=$L/librt_hip$v.so timeout -k 10 300 python3 -u tools/bench_configs.py > $O/configs$v.jsonl 2>> $O/configs.err || exit 1
done
