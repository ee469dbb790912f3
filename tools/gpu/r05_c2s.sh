# Claim-order key from two primary rays per pixel (RT_COST_2S variant) against one, the full C3
# frame and three 8-way shares, alternating
#   gpurun -- 'bash tools/gpu/r05_c2s.sh'
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_c2s; rm -rf $O; mkdir -p $O
RT_HIP_LIB=raytracing-tests_amd/librt_hip_c2s.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py > $O/tests.log 2>&1 || exit 1
B="timeout -k 10 300 python3 bench.py --no-cpu-baseline --config c3"
for i in 1 2; do
  for v in base c2s; do
    X=""; [ $v != base ] && X="RT_HIP_LIB=raytracing-tests_amd/librt_hip_$v.so"
    env $X $B --steps 3 > $O/${v}_full_$i.json 2> $O/${v}_full_$i.err || exit 1
    for r in 0 1 6; do
      env $X RT_BENCH_SHARD=$r/8 $B --steps 5 > $O/${v}_s${r}_$i.json 2> $O/${v}_s${r}_$i.err || exit 1
    done
  done
done
python3 - $O <<'PY'
import json, sys
o = sys.argv[1]
for v in ("base", "c2s"):
    for w in ("full", "s0", "s1", "s6"):
        print(v, w, [json.load(open(f"{o}/{v}_{w}_{i}.json"))["ms_per_step"] for i in (1, 2)])
PY
