set -o pipefail
mkdir -p gpurun_out/probe
timeout -k 10 300 python tools/latency_probe.py > gpurun_out/probe/lat.json 2> gpurun_out/probe/lat.err || exit 1
