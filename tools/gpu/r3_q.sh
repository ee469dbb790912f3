# claim order on pixel-major frames only: full -m gpu suite, C3 / C5 rows
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd "$R"
O=gpurun_out/r3q
rm -rf $O && mkdir -p $O
run() { timeout -k 10 300 python3 tools/bench_configs.py "$@" >> $O/rows.jsonl 2>> $O/rows.err; }
run --row c5 --spp 64 --reps 2 || exit 1
run --row c3 --spp 500 --reps 2 || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || exit 1
