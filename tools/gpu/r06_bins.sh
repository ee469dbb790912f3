# Time-binned culling trees and beam lists (rt_options.inw_time_bins / inw_walk_bins /
# inw_beam_bins): the INW GPU parity tests, then C3 A/B of the settings.
#   gpurun -- 'bash tools/gpu/r06_bins.sh [tests|ab|all]'
set -o pipefail
O=gpurun_out/r06_bins; mkdir -p $O
P=${1:-all}
if [ $P != ab ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_bvh_exact.py > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
  tail -2 $O/gpu_tests.log
fi
if [ $P != tests ]; then
  rm -f $O/*.json
  for i in 1 2; do
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 > $O/def_$i.json 2> $O/def_$i.err || exit 1
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --opt inw_walk_bins=0 > $O/bw4_$i.json 2> $O/bw4_$i.err || exit 1
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --opt inw_time_bins=2 > $O/t2_$i.json 2> $O/t2_$i.err || exit 1
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --opt inw_time_bins=2 --opt inw_walk_bins=0 > $O/bw2_$i.json 2> $O/bw2_$i.err || exit 1
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --opt inw_time_bins=0 > $O/t0_$i.json 2> $O/t0_$i.err || exit 1
  done
fi
echo done
