# Round-6 same-box A/Bs of k_inw_pm's GQ instance, C3 (BASELINE configs[2]) at full size:
# the product (quantised nodes + 1,168 staged + global FStack), inw_qnodes=0 (the round-5 kernel),
# RT_GQ_FSTACK (quantised nodes, LDS FStack, nothing staged), RT_GQ_STAGE=0 (global FStack, nothing
# staged); then the RT_DIAG_OCC build's per-phase lane occupancy (reference-walk fallbacks) of both.
#   gpurun -- 'bash tools/gpu/r06_ab.sh'
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_ab; rm -rf $O; mkdir -p $O
B="timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5"
L=$GRAFT_REPO_ROOT/raytracing-tests_amd
for i in 1 2; do
  $B > $O/gq_$i.json 2> $O/gq_$i.err || exit 1
  $B --opt inw_qnodes=0 > $O/base_$i.json 2> $O/base_$i.err || exit 1
  RT_HIP_LIB=$L/librt_hip_gqf.so $B > $O/gqf_$i.json 2> $O/gqf_$i.err || exit 1
  RT_HIP_LIB=$L/librt_hip_gqns.so $B > $O/gqns_$i.json 2> $O/gqns_$i.err || exit 1
done
RT_HIP_LIB=$L/librt_hip_occ.so timeout -k 10 300 python3 tools/inw_occ.py c3 > $O/occ_gq.json 2> $O/occ_gq.err || exit 1
RT_HIP_LIB=$L/librt_hip_occ.so timeout -k 10 300 python3 tools/inw_occ.py c3 0 inw_qnodes=0 > $O/occ_base.json 2> $O/occ_base.err || exit 1
echo done
