# C5 fold order: the probe's pick (sample-major) against forced pixel-major.
#   gpurun -- 'bash tools/gpu/r06_c5order.sh'
set -o pipefail
O=gpurun_out/r06_c5order; rm -rf $O; mkdir -p $O
timeout -k 10 300 python3 bench.py --config c5 --no-cpu-baseline --steps 1 > $O/sm_1.json 2> $O/sm_1.err || exit 1
timeout -k 10 300 python3 bench.py --config c5 --no-cpu-baseline --steps 1 --opt inw_order=1 > $O/pm_1.json 2> $O/pm_1.err || exit 1
echo done
