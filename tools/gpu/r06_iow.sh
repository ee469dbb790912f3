# Round-6 IOW-03 check after the record layout change (SpecRecs::ix, pixel-major records): the
# IOW-03 GPU tests (oracle parity incl. the full-spp C2 blocks and the strategy matrix), then the C2
# bench line with its kernel trace and PMC passes (tools/gpu/profile.sh c2).
#   gpurun -- 'bash tools/gpu/r06_iow.sh'
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_iow; rm -rf $O; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    -k "iow or IOW or c2 or spec or seeds or progressive or properties" > $O/gpu_tests.log 2>&1 || exit 1
STEPS=3 bash tools/gpu/profile.sh c2 || exit 1
echo done
