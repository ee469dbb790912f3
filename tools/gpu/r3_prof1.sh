# counter list + C3 timing after the issue/wait trims + the c3 profile (kernel trace + PMC)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd "$R"
O=gpurun_out/r3h
rm -rf $O && mkdir -p $O
timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1 || true
timeout -k 10 200 python3 tools/bench_configs.py --row c3 --spp 500 --reps 2 >> $O/rows.jsonl 2>> $O/rows.err || exit 1
bash tools/gpu/profile.sh c3 || exit 1
