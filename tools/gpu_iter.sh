# one GPU iteration: parity tests, then a bench probe (each step time-limited, chained with &&)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -s -p no:cacheprovider > gpurun_out/parity.log 2>&1 && \
timeout -k 10 600 python bench.py ${BENCH_ARGS:---spp 4 --steps 1 --warmup 1 --no-cpu-baseline} > gpurun_out/bench.json 2> gpurun_out/bench.err
