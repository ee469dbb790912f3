# Session probe: smoke on cuda:0, then the single-pixel latency probe (per-segment cycle split)
set -o pipefail
O=gpurun_out/probe3
rm -rf $O && mkdir -p $O
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/latency_probe.py > $O/latency.json 2> $O/latency.err || exit 1
timeout -k 10 400 python3 -u tools/bench_configs.py > $O/configs.jsonl 2> $O/configs.err || exit 1
