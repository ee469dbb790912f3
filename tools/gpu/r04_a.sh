cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04a; rm -rf $O; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_fullspp.py tests/test_gpu_bvh_exact.py -k "fullspp or inw" -x -v -s --timeout 400 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { echo TESTS_FAILED; exit 1; }
timeout -k 10 240 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
