# k_inw_sm's fold ring in LDS (C5): the exactness tests of the fold kernels, then C5 with the LDS
# ring (default) and the global ring of round 4 (inw_ring_sm=256), each with one HBM-traffic PMC pass
#   gpurun -- 'bash tools/gpu/r05_ring.sh'
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_ring; rm -rf $O; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bvh_exact.py tests/test_gpu_parity.py -k "strategies or path or inw04 or repeated" > $O/tests.log 2>&1 || exit 1
B="timeout -k 10 300 python3 bench.py --no-cpu-baseline --config c5"
$B --steps 2 > $O/c5_lds.json 2> $O/c5_lds.err || exit 1
$B --steps 2 --opt inw_ring_sm=256 > $O/c5_global.json 2> $O/c5_global.err || exit 1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE -d $O/pmc_lds -o run --output-format csv -- python3 bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline > $O/pmc_lds.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE -d $O/pmc_global -o run --output-format csv -- python3 bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline --opt inw_ring_sm=256 > $O/pmc_global.log 2>&1 || exit 1
echo done
