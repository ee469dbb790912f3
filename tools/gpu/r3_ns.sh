# north-star 8-way shares: default probe stride (64) against a stride of 8 on every share (the
# share's probe then holds as many pixels as the full frame's)
set -o pipefail
O=gpurun_out/r3ns
rm -rf $O && mkdir -p $O
A="--config ns --steps 1 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 python3 bench.py $A > $O/n1.json 2> $O/n1.err || exit 1
for P in 64 8; do
  for r in 0 1 2 3 4 5 6 7; do
    RT_SPEC_PROBE=$P RT_BENCH_SHARD=$r/8 timeout -k 10 200 python3 bench.py $A > $O/p${P}_s$r.json 2> $O/p${P}_s$r.err || exit 1
  done
done
