# last check of the tree as the driver will run it: smoke, parity tests, a short bench line
set -o pipefail
O=gpurun_out/final
rm -rf $O && mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_stages.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 > $O/bench.json 2> $O/bench.err || exit 1
