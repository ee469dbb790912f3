set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/parity.log 2>&1 || exit 1
B="python bench.py --steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 $B > gpurun_out/fix.json 2> gpurun_out/err.log || exit 1
RT_SPEC_FIX=0 timeout -k 10 300 $B > gpurun_out/nofix.json 2>> gpurun_out/err.log || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_sp -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/kt_sp.log 2>&1
