# Row claims (8 ordinals at a time) against per-pixel claims in k_inw_pm: exactness tests of the
# row build, C3 A/B, and the fold kernel's WRITE_SIZE / FETCH_SIZE for both
#   gpurun -- 'bash tools/gpu/r05_rows.sh'
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_rows; rm -rf $O; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_bvh_exact.py > $O/tests.log 2>&1 || exit 1
bash tools/gpu/r05_ab_variant.sh cpix c3 || exit 1
for v in rows pix; do
  X=""; [ $v = pix ] && X="RT_HIP_LIB=raytracing-tests_amd/librt_hip_cpix.so"
  for c in FETCH_SIZE WRITE_SIZE; do
    env $X timeout -s KILL 300 rocprofv3 --pmc $c -d $O/${v}_$c -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/${v}_$c.log 2>&1 || exit 1
  done
done
echo done
