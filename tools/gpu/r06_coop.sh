# North-star share 3/8 with wider cooperative closest hits (rt_options.iow_coop_max, default 4).
#   gpurun -- 'bash tools/gpu/r06_coop.sh'
set -o pipefail
O=gpurun_out/r06_coop; rm -rf $O; mkdir -p $O
A="--config ns --steps 1 --warmup 1 --no-cpu-baseline"
for c in ${COOPS:-4 8 16 0}; do
  RT_BENCH_SHARD=3/8 timeout -k 10 300 python3 bench.py $A --opt iow_coop_max=$c > $O/coop$c.json 2> $O/coop$c.err || exit 1
done
echo done
