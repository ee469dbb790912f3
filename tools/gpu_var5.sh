# INW 3 vs 4 waves per SIMD (bench_configs), bench frame back on the default build, C4 prediction at 500 spp
set -o pipefail
O=gpurun_out/var5
rm -rf $O && mkdir -p $O
L=raytracing-tests_amd
timeout -k 10 300 python3 -u tools/bench_configs.py --quick > $O/configs_main.jsonl 2> $O/configs.err || exit 1
RT_HIP_LIB=$L/librt_hip_inw4.so timeout -k 10 300 python3 -u tools/bench_configs.py --quick > $O/configs_inw4.jsonl 2>> $O/configs.err || exit 1
timeout -k 10 200 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench.jsonl 2> $O/bench.err || exit 1
timeout -k 10 300 python3 -u tools/c4_scale.py 500 > $O/c4_scale.jsonl 2> $O/c4.err || exit 1
