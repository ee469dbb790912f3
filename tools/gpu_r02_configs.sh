# round 2: smoke, then BASELINE's other configs at full spp on persistent scenes
set -o pipefail
O=gpurun_out/r02cfg
mkdir -p $O
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/bench_configs.py --full --reps 2 > $O/full.jsonl 2> $O/full.err || exit 1
timeout -k 10 300 python -u tools/bench_configs.py > $O/default.jsonl 2> $O/default.err || exit 1
