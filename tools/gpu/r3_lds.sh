# N1: the pixel-major kernel with the top of the wide BVH staged in LDS (RT_INW_LDS=1, 768-lane
# blocks at 3 waves per SIMD) against the default (4 waves per SIMD, nodes from L1/L2)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd "$R"
O=gpurun_out/r3j
rm -rf $O && mkdir -p $O
RT_INW_LDS=1 RT_INW_ORDER=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "inw" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/parity.log 2>&1 || exit 1
run() { timeout -k 10 200 python3 tools/bench_configs.py "$@" >> $O/rows.jsonl 2>> $O/rows.err; }
run --row c3 --spp 500 --reps 2 || exit 1
RT_INW_LDS=1 run --row c3 --spp 500 --reps 2 || exit 1
run --row c3 --spp 64 --reps 2 || exit 1
RT_INW_LDS=1 run --row c3 --spp 64 --reps 2 || exit 1
