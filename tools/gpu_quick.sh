# quick GPU check after a kernel change: parity + strategy exactness tests, then the bench line
# usage: bash tools/gpu_quick.sh TAG [extra pytest -k expr]
set -o pipefail
O=gpurun_out/quick_$1
mkdir -p $O
K=${2:-}
if [ -n "$K" ]; then KA="-k $K"; else KA=""; fi
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bvh_exact.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider $KA > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
python3 -c "import json;d=json.load(open('$O/bench.json'));print('bench', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['counters_per_step'])"
