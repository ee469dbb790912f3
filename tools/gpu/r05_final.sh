# Round-5 evidence on one MI355X: smoke + the -m gpu suite; the C3 bench line with its kernel trace
# and PMC passes; the reference's redraw (--rebuild) with the walk structures built on the device
# and on the host; C5 and C2 bench lines; the fold kernels' lane occupancy per phase (RT_DIAG_OCC
# build, N2); the 8-way C4 shares.
#   gpurun -- 'bash tools/gpu/r05_final.sh check'   (smoke, -m gpu suite, C3 profile)
#   gpurun -- 'bash tools/gpu/r05_final.sh rest'    (the other lines)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
if [ "${1:-check}" = check ]; then
  bash tools/gpu/check.sh || exit 1
  bash tools/gpu/profile.sh c3 || exit 1
  echo done; exit 0
fi
O=gpurun_out/r05_final; rm -rf $O; mkdir -p $O
B="timeout -k 10 400 python3 bench.py --no-cpu-baseline"
$B --steps 5 --rebuild > $O/c3_rebuild_dev.json 2> $O/c3_rebuild_dev.err || exit 1
$B --steps 5 --rebuild --opt inw_device_build=0 > $O/c3_rebuild_host.json 2> $O/c3_rebuild_host.err || exit 1
$B --config c5 --steps 2 > $O/c5.json 2> $O/c5.err || exit 1
$B --config c2 --steps 2 > $O/c2.json 2> $O/c2.err || exit 1
RT_HIP_LIB=raytracing-tests_amd/librt_hip_occ.so timeout -k 10 300 python3 tools/inw_occ.py c3 > $O/occ_c3.txt 2>&1 || exit 1
RT_HIP_LIB=raytracing-tests_amd/librt_hip_occ.so timeout -k 10 300 python3 tools/inw_occ.py c5 > $O/occ_c5.txt 2>&1 || exit 1
bash tools/gpu/shares.sh c3 8 3 > $O/shares_c3.log 2>&1 || exit 1
echo done
