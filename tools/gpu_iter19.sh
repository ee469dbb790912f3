# texture path + new speculation defaults: smoke, the whole GPU suite, a 2-step bench
set -o pipefail
mkdir -p gpurun_out/v19
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v19/smoke.log 2>&1 || exit 1
timeout -k 10 1000 python -m pytest tests -m gpu -q -x -s -p no:cacheprovider > gpurun_out/v19/parity.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/v19/bench.json 2> gpurun_out/v19/bench.err || exit 1
