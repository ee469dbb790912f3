# Round-6 same-box A/Bs of the GQ instance (global 40-float stacks) at C3 full size: quantised vs
# full nodes staged, 3 vs 4 waves per SIMD, buffer-load node fetch (bl), against inw_qnodes=0 (the
# round-5 kernel); then the
# RT_DIAG_OCC build's lane occupancy / reference-walk fallbacks of the product and the round-5 kernel.
#   gpurun -- 'bash tools/gpu/r06_ab2.sh'
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_ab2; rm -rf $O; mkdir -p $O
B="timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5"
L=$GRAFT_REPO_ROOT/raytracing-tests_amd
for i in 1 2; do
  $B --opt inw_qnodes=0 > $O/base_$i.json 2> $O/base_$i.err || exit 1
  $B --opt inw_qnodes=1 > $O/q3_$i.json 2> $O/q3_$i.err || exit 1
  for v in f3 f4 q4 bl; do
    RT_HIP_LIB=$L/librt_hip_$v.so $B $( [ $v = bl ] && echo --opt inw_qnodes=0 ) > $O/${v}_$i.json 2> $O/${v}_$i.err || exit 1
  done
done
RT_HIP_LIB=$L/librt_hip_occ.so timeout -k 10 300 python3 tools/inw_occ.py c3 > $O/occ_q3.json 2> $O/occ_q3.err || exit 1
RT_HIP_LIB=$L/librt_hip_occ.so timeout -k 10 300 python3 tools/inw_occ.py c3 0 inw_qnodes=0 > $O/occ_base.json 2> $O/occ_base.err || exit 1
echo done
