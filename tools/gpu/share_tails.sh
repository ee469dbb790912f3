# 8-way share tails: the phase-split timeline of shares 0/8 and 6/8 with the default claim-order
# estimate (16 pixels per block), every pixel of the block (RT_COST64 build) and unit order
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/share_tails; rm -rf $O; mkdir -p $O
L=$GRAFT_REPO_ROOT/raytracing-tests_amd
for sh in 0/8 6/8; do
  t=$(echo $sh | tr '/' 'o')
  RT_HIP_LIB=$L/librt_hip_split.so timeout -k 10 200 python3 tools/inw_split.py c3 500 $sh > $O/split_$t.json 2>> $O/err.txt || exit 1
  RT_HIP_LIB=$L/librt_hip_c64s.so timeout -k 10 200 python3 tools/inw_split.py c3 500 $sh > $O/split_c64_$t.json 2>> $O/err.txt || exit 1
  RT_HIP_LIB=$L/librt_hip_split.so timeout -k 10 200 python3 tools/inw_split.py c3 500 $sh inw_claim_order=0 > $O/split_nocost_$t.json 2>> $O/err.txt || exit 1
done
RT_HIP_LIB=$L/librt_hip_c64s.so timeout -k 10 200 python3 tools/inw_split.py c3 500 > $O/split_c64_full.json 2>> $O/err.txt || exit 1
