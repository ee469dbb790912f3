# round 2: the prior-only guess (RT_SPEC_PRIOR_S0=0) -- exactness, 1-GPU bench, 8-way shard prediction
set -o pipefail
O=gpurun_out/r02prior
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_bvh_exact.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
RT_SPEC_PRIOR_S0=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_s0.json 2> $O/bench_s0.err || exit 1
bash tools/gpu_shard.sh 8 || exit 1
cp gpurun_out/shard/b8_*.json $O/
