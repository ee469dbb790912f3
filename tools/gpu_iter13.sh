set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/parity.log 2>&1 || exit 1
B="python bench.py --steps 1 --warmup 0 --no-cpu-baseline"
for g in 4 8 2; do
  RT_SPEC_GROUPS=$g timeout -k 10 300 $B > gpurun_out/g_$g.json 2>> gpurun_out/err.log || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_sp -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/kt_sp.log 2>&1
