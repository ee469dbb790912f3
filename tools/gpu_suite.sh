# smoke + the whole GPU suite
set -o pipefail
mkdir -p gpurun_out/suite
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/suite/smoke.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/suite/gpu_tests.log 2>&1 || exit 1
