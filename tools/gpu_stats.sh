set -o pipefail
mkdir -p gpurun_out/stats
RT_SPEC_ITERS=1 timeout -k 10 300 python tools/spec_stats.py > gpurun_out/stats/stats.json 2> gpurun_out/stats/stats.err || exit 1
RT_SPEC_ROUNDS=32 timeout -k 10 300 python tools/spec_stats.py > gpurun_out/stats/stats32.json 2>> gpurun_out/stats/stats.err || exit 1
