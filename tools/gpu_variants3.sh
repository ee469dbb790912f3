# Variant builds (make variant): lone-pixel probe per build, then the bench frame per build
set -o pipefail
O=gpurun_out/var3
rm -rf $O && mkdir -p $O
L=raytracing-tests_amd
for v in diag diagm; do
  RT_HIP_LIB=$L/librt_hip_$v.so timeout -k 10 200 python3 -u tools/variant_probe.py > $O/probe_$v.json 2> $O/probe_$v.err || exit 1
done
for v in "" _merge "" _merge; do
  RT_HIP_LIB=$L/librt_hip$v.so timeout -k 10 200 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline >> $O/bench$v.jsonl 2>> $O/bench.err || exit 1
done
