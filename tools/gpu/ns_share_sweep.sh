# North-star (IOW-03 final scene, 1920x1080, 500 spp) share sensitivity: one 8-way share rendered
# alone per IOW-03 option setting (the heaviest share of profiles/r03_ns_shares_heavy48.json is 6/8).
#   gpurun -- 'SHARE=6 bash tools/gpu/ns_share_sweep.sh "spec_tail_budget=1536" "spec_tail_rounds=30" ...'
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/ns_sweep; rm -rf $O; mkdir -p $O
S=${SHARE:-6}
A="--config ns --steps 1 --warmup 1 --no-cpu-baseline"
i=0
for setting in default "$@"; do
  i=$((i+1))
  X=""
  if [ "$setting" != default ]; then for kv in $setting; do X="$X --opt $kv"; done; fi
  RT_BENCH_SHARD=$S/8 timeout -k 10 300 python3 bench.py $A $X > $O/s$i.json 2> $O/s$i.err || exit 1
  python3 -c "import json,sys; b=json.load(open('$O/s$i.json')); print('$setting', b['ms_per_step'], b['roofline']['main_kernel_ms_per_frame'], b['roofline']['launches_per_frame'])"
done
