# A/B of library variants on one box: the INW parity cases on the default build, then
# `bench.py --config CFG` for each variant (raytracing-tests_amd/librt_hip<suffix>.so, "-" = the
# default build), in two interleaved passes so that box drift hits every variant alike.
#   gpurun -- 'bash tools/gpu/ab.sh c3 "- _base -:inw_beams=0"'
set -o pipefail
CFG=${1:-c3}
VARS=${2:--}
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd "$R"
O=gpurun_out/ab
rm -rf $O && mkdir -p $O
if [ -z "$NOPARITY" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "inw" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/parity_inw.log 2>&1 || exit 1
fi
# a variant is SUFFIX or SUFFIX:FIELD=VAL[:FIELD=VAL...] (rt_options fields for that run only)
for pass in 1 2; do
  for v in $VARS; do
    IFS=: read -r s envs <<< "$v"
    [ "$s" = "-" ] && s=""
    tag=${CFG}${s}$(echo "$envs" | tr -c 'A-Za-z0-9_\n' '_')
    opts=""
    for kv in $(echo "$envs" | tr ':' ' '); do opts="$opts --opt $kv"; done
    RT_HIP_LIB=$R/raytracing-tests_amd/librt_hip$s.so timeout -k 10 200 python3 bench.py --config $CFG --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline $opts > $O/${tag}_p$pass.json 2> $O/${tag}_p$pass.err || exit 1
  done
done
python3 - $O <<'PY'
import json, glob, sys, os
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    b = json.load(open(f))
    print(os.path.basename(f), b["ms_per_step"], b["roofline"]["kernel"], round(b["roofline"]["avg_launch_ms"], 2))
PY
