# round-end evidence, part 3: BASELINE's other configs at full spp and the C4 prediction
set -o pipefail
O=gpurun_out/round
mkdir -p $O
timeout -k 10 400 python3 -u tools/bench_configs.py --full > $O/configs_full.jsonl 2> $O/configs_full.err || exit 1
timeout -k 10 300 python3 -u tools/c4_scale.py 500 > $O/c4_scale.jsonl 2> $O/c4.err || exit 1
