# fold-window size of k_inw_o on C5 / C3, against the record path
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd "$R"
O=gpurun_out/r3e
rm -rf $O && mkdir -p $O
run() { timeout -k 10 200 python3 tools/bench_configs.py "$@" >> $O/rows.jsonl 2>> $O/rows.err; }
run --row c5 --spp 16 --reps 2 || exit 1
RT_INW_RING=1024 run --row c5 --spp 16 --reps 2 || exit 1
RT_INW_RING=4096 run --row c5 --spp 16 --reps 2 || exit 1
RT_INW_RING=16384 run --row c5 --spp 16 --reps 2 || exit 1
RT_INW_ORDER=0 run --row c5 --spp 16 --reps 2 || exit 1
RT_INW_RING=1024 run --row c3 --spp 500 --reps 2 || exit 1
RT_INW_RING=4096 run --row c3 --spp 500 --reps 2 || exit 1
RT_INW_RING=4096 run --row c5 --spp 128 --reps 1 || exit 1
RT_INW_ORDER=0 run --row c5 --spp 128 --reps 1 || exit 1
