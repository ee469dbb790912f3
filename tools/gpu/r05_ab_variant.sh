# Same-box A/B of the product library against a variant build (RT_HIP_LIB), C3 frames, alternating
#   gpurun -- 'bash tools/gpu/r05_ab_variant.sh nolds [config]'
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
V=$1; CFG=${2:-c3}
O=gpurun_out/r05_ab_${V}_$CFG; rm -rf $O; mkdir -p $O
B="timeout -k 10 300 python3 bench.py --no-cpu-baseline --config $CFG --steps ${STEPS:-5}"
for i in 1 2; do
  $B > $O/base_$i.json 2> $O/base_$i.err || exit 1
  RT_HIP_LIB=raytracing-tests_amd/librt_hip_$V.so $B > $O/var_$i.json 2> $O/var_$i.err || exit 1
done
python3 - $O <<'PY'
import json, sys
o = sys.argv[1]
for n in ("base_1", "var_1", "base_2", "var_2"):
    d = json.load(open(f"{o}/{n}.json"))
    print(n, d["ms_per_step"], d["roofline"]["main_kernel_ms_per_frame"], d.get("parity", {}).get("exact_frac") if d.get("parity") else None)
PY
