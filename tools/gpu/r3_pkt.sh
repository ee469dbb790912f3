# wave-packet walk (RT_INW_PACKET=1): parity and C3 / C5 timing against the per-lane wide walk
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd "$R"
O=gpurun_out/r3i
rm -rf $O && mkdir -p $O
RT_INW_PACKET=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "inw or tile_list" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/parity.log 2>&1 || exit 1
run() { timeout -k 10 200 python3 tools/bench_configs.py "$@" >> $O/rows.jsonl 2>> $O/rows.err; }
run --row c3 --spp 500 || exit 1
RT_INW_PACKET=1 run --row c3 --spp 500 || exit 1
run --row c5 --spp 64 || exit 1
RT_INW_PACKET=1 run --row c5 --spp 64 || exit 1
RT_INW_PACKET=1 RT_INW_ORDER=2 run --row c3 --spp 500 || exit 1
