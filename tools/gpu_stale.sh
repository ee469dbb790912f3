set -o pipefail
mkdir -p gpurun_out/stale
RT_DEBUG_FIRST_STALE=1 RT_SPEC_HEAVY=5 timeout -k 10 300 python tools/spec_stats.py > gpurun_out/stale/stats.json 2> gpurun_out/stale/stats.err || exit 1
