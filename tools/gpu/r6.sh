# A/B of library variants on C3 + the phase split / timeline of one 8-way share
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6; rm -rf $O; mkdir -p $O
NOPARITY=1 bash tools/gpu/ab.sh c3 "${VARS:-- _pf}" > $O/ab.txt 2>&1 || exit 1
RT_HIP_LIB=$GRAFT_REPO_ROOT/raytracing-tests_amd/librt_hip_split.so timeout -k 10 200 python3 tools/inw_split.py c3 500 0/8 > $O/split_c3_s0of8.json 2> $O/split.err || exit 1
RT_HIP_LIB=$GRAFT_REPO_ROOT/raytracing-tests_amd/librt_hip_split.so timeout -k 10 200 python3 tools/inw_split.py c3 500 > $O/split_c3.json 2>> $O/split.err || exit 1
