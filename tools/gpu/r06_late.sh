# Round-6 late evidence: phase splits of C3 and C5 on the final code, the time-bin count again
# with compact nodes, and the C3 8-way shares.
#   gpurun -- 'bash tools/gpu/r06_late.sh'
set -o pipefail
O=gpurun_out/r06_late; rm -rf $O; mkdir -p $O
L=$GRAFT_REPO_ROOT/raytracing-tests_amd
RT_HIP_LIB=$L/librt_hip_split.so timeout -k 10 300 python3 tools/inw_split.py c3 > $O/split_c3.json 2> $O/split.err || exit 1
RT_HIP_LIB=$L/librt_hip_split.so timeout -k 10 300 python3 tools/inw_split.py c5 > $O/split_c5.json 2>> $O/split.err || exit 1
for i in 1 2; do
  for b in 2 3; do
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --opt inw_time_bins=$b > $O/t${b}_$i.json 2> $O/t${b}_$i.err || exit 1
  done
done
bash tools/gpu/shares.sh c3 8 3 > $O/shares_c3.log 2>&1 || exit 1
echo done
