# INW parity (wide walk guard, RI-walk skip) + C3 A/B of record-store variants
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd "$R"
O=gpurun_out/r3b
rm -rf $O && mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "inw" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/parity_inw.log 2>&1 || exit 1
for v in "" _nt _norec; do
  RT_HIP_LIB=$R/raytracing-tests_amd/librt_hip$v.so timeout -k 10 200 python3 bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/c3$v.json 2> $O/c3$v.err || exit 1
done
