# Round-6 IOW-03 walk: the octant near/far cull (cull4o, product) against the pair form
# (RT_IOW_NO_OCTANT): the IOW-03 GPU tests, then C2 same-box A/B.
#   gpurun -- 'bash tools/gpu/r06_iow2.sh'
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_iow2; rm -rf $O; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    -k "iow or IOW or c2 or spec or seeds or progressive or properties" > $O/gpu_tests.log 2>&1 || exit 1
B="timeout -k 10 300 python3 bench.py --config c2 --no-cpu-baseline --steps 3"
for i in 1 2; do
  $B > $O/oct_$i.json 2> $O/oct_$i.err || exit 1
  RT_HIP_LIB=$GRAFT_REPO_ROOT/raytracing-tests_amd/librt_hip_noct.so $B > $O/noct_$i.json 2> $O/noct_$i.err || exit 1
done
echo done
