# Device build of the per-redraw walk structures: the update tests (fresh scene against updated
# scene, device build against host build), then the update timing and its kernel trace.
#   gpurun -- 'bash tools/gpu/r05_build.sh'
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_build; rm -rf $O; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_lbvh.py -k "update or iow03_tile or lbvh" > $O/tests.log 2>&1 || exit 1
timeout -k 10 120 python3 tools/prof_update.py 20 1 > $O/dev.json 2> $O/dev.err || exit 1
timeout -k 10 120 python3 tools/prof_update.py 5 0 > $O/host.json 2> $O/host.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 tools/prof_update.py 20 1 > $O/kt.log 2>&1 || exit 1
echo done
