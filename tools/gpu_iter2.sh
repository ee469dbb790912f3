# parity (all gpu tests) -> bench probe -> one PMC pass for VALU lane utilisation
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof2
timeout -k 10 900 python -m pytest tests -m gpu -q -s -p no:cacheprovider > gpurun_out/parity.log 2>&1
timeout -k 10 600 python bench.py ${BENCH_ARGS:---spp 4 --steps 1 --warmup 1 --no-cpu-baseline} > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES -d gpurun_out/prof2/pmc -o run --output-format csv -- python3 bench.py --spp 2 --width 600 --height 400 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/prof2/pmc.log 2>&1
