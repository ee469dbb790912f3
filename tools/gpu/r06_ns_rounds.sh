# North-star 8-way share 3/8 (the slowest in profiles/r06_shares_ns_8.json) rendered alone under
# the speculation's round options: do fixed per-launch drain tails explain the shares' overhead?
#   gpurun -- 'bash tools/gpu/r06_ns_rounds.sh'
set -o pipefail
O=gpurun_out/r06_ns_rounds; rm -rf $O; mkdir -p $O
A="--config ns --steps 1 --warmup 1 --no-cpu-baseline"
run() {  # name, bench args
  local n=$1; shift
  RT_BENCH_SHARD=3/8 timeout -k 10 300 python3 bench.py $A "$@" > $O/$n.json 2> $O/$n.err || exit 1
}
run def
run r12 --opt spec_rounds=12
run r6 --opt spec_rounds=6
run t30 --opt spec_tail_rounds=30
run b8k --opt spec_tail_budget=8192
run r12t30 --opt spec_rounds=12 --opt spec_tail_rounds=30
echo done
