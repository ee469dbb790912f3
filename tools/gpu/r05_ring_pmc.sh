# HBM traffic of C5 with k_inw_sm's LDS ring (default) and the global ring (inw_ring_sm=256):
# FETCH_SIZE and WRITE_SIZE in passes of their own
#   gpurun -- 'bash tools/gpu/r05_ring_pmc.sh'
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_ring_pmc; rm -rf $O; mkdir -p $O
for v in lds global; do
  X=""; [ $v = global ] && X="--opt inw_ring_sm=256"
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $c -d $O/${v}_$c -o run --output-format csv -- python3 bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline $X > $O/${v}_$c.log 2>&1 || exit 1
  done
done
echo done
