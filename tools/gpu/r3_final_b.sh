# the C3 profile again (the previous copy-back overflowed) + the INW phase split (diagnostic build)
set -o pipefail
bash tools/gpu/profile.sh c3 || exit 1
RT_HIP_LIB=$GRAFT_REPO_ROOT/raytracing-tests_amd/librt_hip_split.so timeout -k 10 200 python3 tools/inw_split.py c3 > gpurun_out/split_c3.json 2>&1 || exit 1
RT_HIP_LIB=$GRAFT_REPO_ROOT/raytracing-tests_amd/librt_hip_split.so timeout -k 10 200 python3 tools/inw_split.py c5 64 > gpurun_out/split_c5.json 2>&1 || exit 1
