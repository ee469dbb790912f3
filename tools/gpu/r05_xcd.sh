# Per-XCD claim queues of k_inw_pm (inw_claim_xcd=1, default) against one queue: exactness tests,
# C3 frames of both, and the fold kernel traffic (FETCH_SIZE, WRITE_SIZE in passes of their own)
#   gpurun -- 'bash tools/gpu/r05_xcd.sh'
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_xcd; rm -rf $O; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_bvh_exact.py tests/test_gpu_parity.py tests/test_gpu_fullspp.py -k "strategies or render_matches_oracle or c3_full" > $O/tests.log 2>&1 || exit 1
B="timeout -k 10 300 python3 bench.py --no-cpu-baseline"
$B --steps 5 > $O/c3_xq.json 2> $O/c3_xq.err || exit 1
$B --steps 5 --opt inw_claim_xcd=0 > $O/c3_one.json 2> $O/c3_one.err || exit 1
for v in xq one; do
  X=""; [ $v = one ] && X="--opt inw_claim_xcd=0"
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $c -d $O/${v}_$c -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline $X > $O/${v}_$c.log 2>&1 || exit 1
  done
done
echo done
