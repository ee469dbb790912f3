# k_inw_o (wave-ordered INW): parity vs oracle, C3 bench against the records path
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd "$R"
O=gpurun_out/r3c
rm -rf $O && mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "inw or tile_list" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/parity_inw.log 2>&1 || exit 1
timeout -k 10 200 python3 bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/c3_ord.json 2> $O/c3_ord.err || exit 1
RT_INW_ORDER=0 timeout -k 10 200 python3 bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/c3_rec.json 2> $O/c3_rec.err || exit 1
timeout -k 10 300 python3 tools/bench_configs.py --quick > $O/configs_quick.jsonl 2> $O/configs_quick.err || exit 1
