set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python tools/bench_configs.py > gpurun_out/configs.jsonl 2> gpurun_out/err.log
