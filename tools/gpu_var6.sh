# id-dirs reuse in the cooperative segment (lone split + bench), INW-01 at 4 waves per SIMD (configs)
set -o pipefail
O=gpurun_out/var6
rm -rf $O && mkdir -p $O
L=raytracing-tests_amd
for v in diag diagidd; do
  RT_HIP_LIB=$L/librt_hip_$v.so timeout -k 10 200 python3 -u tools/variant_probe.py > $O/probe_$v.json 2> $O/probe_$v.err || exit 1
done
for v in "" _idd "" _idd; do
  RT_HIP_LIB=$L/librt_hip$v.so timeout -k 10 200 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline >> $O/bench$v.jsonl 2>> $O/bench.err || exit 1
done
timeout -k 10 300 python3 -u tools/bench_configs.py > $O/configs_main.jsonl 2> $O/configs.err || exit 1
RT_HIP_LIB=$L/librt_hip_inw4.so timeout -k 10 300 python3 -u tools/bench_configs.py > $O/configs_inw4.jsonl 2>> $O/configs.err || exit 1
