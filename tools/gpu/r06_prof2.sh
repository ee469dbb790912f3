# Round-6 re-profiles after the beam scalar loads (C3) and the IOW octant cull (C2), plus the C3
# phase split with the per-round wave cycles.
#   gpurun -- 'bash tools/gpu/r06_prof2.sh c3'   (c3 | c2 | ns)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
case ${1:-c3} in
  c3) bash tools/gpu/profile.sh c3 || exit 1
      RT_HIP_LIB=$GRAFT_REPO_ROOT/raytracing-tests_amd/librt_hip_split.so timeout -k 10 300 python3 tools/inw_split.py c3 > gpurun_out/r06_split2_c3.json 2> gpurun_out/r06_split2_c3.err || exit 1 ;;
  c2) STEPS=3 bash tools/gpu/profile.sh c2 || exit 1 ;;
  ns) STEPS=1 bash tools/gpu/profile.sh ns || exit 1 ;;
esac
echo done
