# Round-6 same-box A/Bs at C3 full size: the buffer-load node fetch (product) against the pointer
# form (nobl), the culling planes with the reference's reciprocals (idc), and the bounce-walk fill
# (round 1 waits for 32 / 48 lanes with a ray: r32 / r48), leaf batches once 32 / 48 lanes hold a leaf
# (lb32 / lb48).
#   gpurun -- 'bash tools/gpu/r06_ab3.sh'
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_ab3; rm -rf $O; mkdir -p $O
B="timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5"
L=$GRAFT_REPO_ROOT/raytracing-tests_amd
for i in 1 2; do
  $B > $O/bl_$i.json 2> $O/bl_$i.err || exit 1
  for v in nobl idc r32 r48 lb32 lb48; do
    RT_HIP_LIB=$L/librt_hip_$v.so $B > $O/${v}_$i.json 2> $O/${v}_$i.err || exit 1
  done
done
echo done
