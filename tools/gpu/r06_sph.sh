# Sphere records (rt_options.inw_sphere_records): the INW GPU parity tests, then C3 A/B.
#   gpurun -- 'bash tools/gpu/r06_sph.sh [tests|ab|all]'
set -o pipefail
O=gpurun_out/r06_sph; mkdir -p $O
P=${1:-all}
if [ $P != ab ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_bvh_exact.py > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
  tail -2 $O/gpu_tests.log
fi
if [ $P != tests ]; then
  rm -f $O/*.json
  for i in 1 2; do
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 > $O/sph_$i.json 2> $O/sph_$i.err || exit 1
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --opt inw_sphere_records=0 > $O/rec_$i.json 2> $O/rec_$i.err || exit 1
  done
fi
echo done
