# Walk-parking threshold A/B (RT_INW_PARK_LANES 5 / 8 (product) / 12 / 16) on C3 frames, alternating
#   gpurun -- 'bash tools/gpu/r05_park.sh'
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_park; rm -rf $O; mkdir -p $O
B="timeout -k 10 300 python3 bench.py --no-cpu-baseline --config c3 --steps 4"
for i in 1 2; do
  for v in base pk5 pk12 pk16; do
    X=""; [ $v != base ] && X="RT_HIP_LIB=raytracing-tests_amd/librt_hip_$v.so"
    env $X $B > $O/${v}_$i.json 2> $O/${v}_$i.err || exit 1
  done
done
python3 - $O <<'PY'
import json, sys
o = sys.argv[1]
for v in ("base", "pk5", "pk12", "pk16"):
    print(v, [json.load(open(f"{o}/{v}_{i}.json"))["ms_per_step"] for i in (1, 2)])
PY
