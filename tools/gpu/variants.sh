# INW parity + exactness on library variants, then the C3 A/B of all of them against the default
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/variants; rm -rf $O; mkdir -p $O
VS=${VS:-_nw _fu4}
for L in $VS; do
  RT_HIP_LIB=$GRAFT_REPO_ROOT/raytracing-tests_amd/librt_hip$L.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bvh_exact.py -k inw -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests$L.log 2>&1 || exit 1
done
NOPARITY=1 bash tools/gpu/ab.sh c3 "- $VS" > $O/ab.txt 2>&1 || exit 1
