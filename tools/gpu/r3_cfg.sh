# C3 / C5 at reduced and full spp: wave-ordered INW kernel (default) vs the record path
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd "$R"
O=gpurun_out/r3d
rm -rf $O && mkdir -p $O
timeout -k 10 300 python3 tools/bench_configs.py > $O/cfg_ord.jsonl 2> $O/cfg_ord.err || exit 1
RT_INW_ORDER=0 timeout -k 10 300 python3 tools/bench_configs.py > $O/cfg_rec.jsonl 2> $O/cfg_rec.err || exit 1
timeout -k 10 300 python3 tools/bench_configs.py --full --inw-only > $O/full_ord.jsonl 2> $O/full_ord.err || exit 1
