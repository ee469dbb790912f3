# Compact 7-float4 nodes (rt_options.inw_compact_nodes): the INW GPU parity tests, then A/B on C3
# and C5.   gpurun -- 'bash tools/gpu/r06_cn.sh [tests|ab|all]'
set -o pipefail
O=gpurun_out/r06_cn; mkdir -p $O
P=${1:-all}
if [ $P != ab ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_bvh_exact.py > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
  tail -2 $O/gpu_tests.log
fi
if [ $P != tests ]; then
  rm -f $O/*.json
  for i in 1 2; do
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 > $O/cn_$i.json 2> $O/cn_$i.err || exit 1
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --opt inw_compact_nodes=0 > $O/n10_$i.json 2> $O/n10_$i.err || exit 1
  done
  timeout -k 10 300 python3 bench.py --config c5 --no-cpu-baseline --steps 1 > $O/c5cn_1.json 2> $O/c5cn_1.err || exit 1
  timeout -k 10 300 python3 bench.py --config c5 --no-cpu-baseline --steps 1 --opt inw_compact_nodes=0 > $O/c5n10_1.json 2> $O/c5n10_1.err || exit 1
fi
echo done
