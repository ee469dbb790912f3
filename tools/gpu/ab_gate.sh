# A/B with parity gates: the INW parity + exactness cases on each library variant listed in GATE
# (suffixes of raytracing-tests_amd/librt_hip_<suffix>.so), then tools/gpu/ab.sh over VARS.
#   gpurun -- 'GATE="unode" bash tools/gpu/ab_gate.sh c3 "- _unode"'
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab_gate
for v in $GATE; do
  RT_HIP_LIB=$GRAFT_REPO_ROOT/raytracing-tests_amd/librt_hip_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bvh_exact.py -k "inw" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_gate/gate_$v.log 2>&1 || { echo GATE_${v}_FAILED; tail -5 gpurun_out/ab_gate/gate_$v.log; exit 1; }
  tail -1 gpurun_out/ab_gate/gate_$v.log
done
NOPARITY=1 bash tools/gpu/ab.sh "$@"
