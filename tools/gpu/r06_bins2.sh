# Time-bin counts again with the sphere records (their smaller object footprint leaves L2 room).
#   gpurun -- 'bash tools/gpu/r06_bins2.sh'
set -o pipefail
O=gpurun_out/r06_bins2; rm -rf $O; mkdir -p $O
for i in 1 2; do
  for b in 0 2 3 4; do
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --opt inw_time_bins=$b > $O/t${b}_$i.json 2> $O/t${b}_$i.err || exit 1
  done
done
echo done
