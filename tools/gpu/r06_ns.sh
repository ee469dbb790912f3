# Round-6 north-star and scaling evidence: the ns profile (bench line, kernel trace, PMC passes of
# k_iow03sL at 1920x1080x500 after the record-layout change), the 8-way shares of ns and C3 rendered
# alone (predicted 8-GPU speed-up), and the C3 phase split (RT_DIAG_SPLIT).
#   gpurun -- 'bash tools/gpu/r06_ns.sh [part]'     part: prof | shares (+ the beam scalar-load A/B)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
if [ "${1:-prof}" = prof ]; then
  STEPS=1 bash tools/gpu/profile.sh ns || exit 1
else
  bash tools/gpu/shares.sh ns 8 1 > gpurun_out/shares_ns.log 2>&1 || exit 1
  bash tools/gpu/shares.sh c3 8 3 > gpurun_out/shares_c3.log 2>&1 || exit 1
  RT_HIP_LIB=$GRAFT_REPO_ROOT/raytracing-tests_amd/librt_hip_split.so timeout -k 10 300 python3 tools/inw_split.py c3 > gpurun_out/r06_split_c3.json 2> gpurun_out/r06_split_c3.err || exit 1
  O=gpurun_out/r06_ab4; rm -rf $O; mkdir -p $O
  for i in 1 2; do
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 > $O/prod_$i.json 2> $O/prod_$i.err || exit 1
    RT_HIP_LIB=$GRAFT_REPO_ROOT/raytracing-tests_amd/librt_hip_bs.so timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 > $O/bs_$i.json 2> $O/bs_$i.err || exit 1
    RT_HIP_LIB=$GRAFT_REPO_ROOT/raytracing-tests_amd/librt_hip_il.so timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 > $O/il_$i.json 2> $O/il_$i.err || exit 1
  done
fi
echo done
