set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/parity.log 2>&1 || exit 1
B="python bench.py --steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 $B > gpurun_out/async.json 2> gpurun_out/err.log || exit 1
timeout -k 10 300 $B --occupancy > gpurun_out/async_occ.json 2>> gpurun_out/err.log || exit 1
