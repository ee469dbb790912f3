# Round-end evidence, part 1: smoke() and the whole -m gpu suite on one MI355X.
#   gpurun -- 'bash tools/gpu/check.sh'
set -o pipefail
O=gpurun_out/check
rm -rf $O && mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || exit 1
tail -3 $O/gpu_tests.log
