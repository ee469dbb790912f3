# C3 at full spp through the single call under INW strategy switches (DESIGN "Other configs")
set -o pipefail
O=gpurun_out/c3probe
mkdir -p $O
for v in "" "RT_INW_SPEC=0" "RT_SPEC_MAX_GB=8" "RT_SPEC_MAX_GB=2"; do
  timeout -k 10 120 env $v python -c "
import sys, json; sys.path[:0]=['.','raytracing-tests_amd','tools']
import rt_amd as R, bench_configs as B
print(json.dumps({'env': '$v', **B.run('C3 full', R.PRESET_INW01_RANDOM, 1234, 10_000, spp=500)}), flush=True)
" >> $O/probe.jsonl 2>> $O/probe.err || exit 1
done
