# Round-4 A/B: two rounds per iteration (primary, then bounce rays) with / without walk parking.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_two; rm -rf $O; mkdir -p $O
L=$GRAFT_REPO_ROOT/raytracing-tests_amd
for v in ${GATES:-two twopark}; do
  RT_HIP_LIB=$L/librt_hip_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bvh_exact.py -k "inw" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/gate_$v.log 2>&1 || { echo GATE_${v}_FAILED; exit 1; }
done
A="--steps 5 --warmup 1 --no-cpu-baseline"
for pass in 1 2; do
  for v in ${VARS:-base park two twopark}; do
    LIB=$L/librt_hip_$v.so; [ $v = base ] && LIB=$L/librt_hip.so
    RT_HIP_LIB=$LIB timeout -k 10 200 python3 bench.py $A > $O/b_${v}_p$pass.json 2> $O/b_${v}_p$pass.err || exit 1
  done
done
RT_HIP_LIB=$L/librt_hip_occtwo.so timeout -k 10 200 python3 tools/inw_occ.py c3 > $O/occ_c3.json 2> $O/occ_c3.err || exit 1
python3 - $O <<'PY'
import json, glob, sys, os
for f in sorted(glob.glob(sys.argv[1] + "/b_*.json")):
    b = json.load(open(f))
    print(os.path.basename(f), b["ms_per_step"], b["roofline"]["avg_launch_ms"])
PY
