# Round-5 same-box A/Bs: the IOW-03 BVH-stack layout (C2: [slot pair][lane][2] against the round-4
# [slot][lane] build, librt_hip_bflat.so), and the reference-walk mode's stack against stackless
# walks, both in the 768-lane instances (C3 at 64 spp, both fold orders).
#   gpurun -- 'bash tools/gpu/r05_ab.sh'
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_ab; rm -rf $O; mkdir -p $O
B="timeout -k 10 300 python3 bench.py --no-cpu-baseline"
FLAT=$GRAFT_REPO_ROOT/raytracing-tests_amd/librt_hip_bflat.so
for i in 1 2; do
  $B --config c2 --steps 3 > $O/c2_pair_$i.json 2> $O/c2_pair_$i.err || exit 1
  RT_HIP_LIB=$FLAT $B --config c2 --steps 3 > $O/c2_flat_$i.json 2> $O/c2_flat_$i.err || exit 1
done
for ord in 1 2; do
  for sl in 1 0; do
    $B --steps 2 --spp 64 --opt inw_wide_walk=0 --opt inw_stackless=$sl --opt inw_order=$ord > $O/c3ref_o${ord}_sl$sl.json 2> $O/c3ref_o${ord}_sl$sl.err || exit 1
  done
done
$B --steps 5 > $O/c3.json 2> $O/c3.err || exit 1
echo done
