# smoke + the whole GPU suite + the default bench line
set -o pipefail
O=gpurun_out/check
mkdir -p $O
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
