# parity (incl. sample-parallel strategies), then bench default + diagnostics
set -o pipefail
mkdir -p gpurun_out
B="python bench.py --steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/parity.log 2>&1 || exit 1
timeout -k 10 300 $B > gpurun_out/sp.json 2> gpurun_out/err.log || exit 1
timeout -k 10 300 $B --occupancy > gpurun_out/sp_occ.json 2>> gpurun_out/err.log || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_sp -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/kt_sp.log 2>&1
