# fold prefetch reverted + fused cull: parity, exactness, C3/C5 timing; C4 shares; IOW lane occupancy
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd "$R"
O=gpurun_out/r3m
rm -rf $O && mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "inw or tile_list" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/parity.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_bvh_exact.py -k "inw" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/exact_inw.log 2>&1 || exit 1
run() { timeout -k 10 300 python3 tools/bench_configs.py "$@" >> $O/rows.jsonl 2>> $O/rows.err; }
run --row c3 --spp 500 --reps 2 || exit 1
RT_INW_FMA=0 run --row c3 --spp 500 --reps 2 || exit 1
run --row c5 --spp 64 --reps 2 || exit 1
timeout -k 10 300 python3 bench.py --config c2 --steps 1 --warmup 1 --no-cpu-baseline --occupancy > $O/c2_occ.json 2> $O/c2_occ.err || exit 1
bash tools/gpu/shares.sh c3 8 3 > $O/shares.log 2>&1 || exit 1
