# k_inw_b (block-ordered, lane-parallel folds): parity at chunk 1 and 64, timing over chunk sizes
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd "$R"
O=gpurun_out/r3f
rm -rf $O && mkdir -p $O
RT_INW_ORDER=2 RT_INW_LCHUNK=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "inw or tile_list" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/parity_b0.log 2>&1 || exit 1
RT_INW_ORDER=2 RT_INW_LCHUNK=6 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "inw or tile_list" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/parity_b6.log 2>&1 || exit 1
RT_INW_ORDER=2 RT_INW_LCHUNK=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "inw_random_spp37 or inw04_cornell or touching" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/parity_b2.log 2>&1 || exit 1
run() { timeout -k 10 200 python3 tools/bench_configs.py "$@" >> $O/rows.jsonl 2>> $O/rows.err; }
for lc in 0 2 4 6; do
  RT_INW_ORDER=2 RT_INW_LCHUNK=$lc run --row c3 --spp 500 || exit 1
  RT_INW_ORDER=2 RT_INW_LCHUNK=$lc run --row c5 --spp 64 || exit 1
done
RT_INW_ORDER=2 RT_INW_LCHUNK=0 RT_INW_RING=1024 run --row c5 --spp 64 || exit 1
RT_INW_ORDER=2 RT_INW_LCHUNK=6 RT_INW_RING=1024 run --row c3 --spp 500 || exit 1
RT_INW_ORDER=0 run --row c5 --spp 64 || exit 1
