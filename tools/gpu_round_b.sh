# round-end evidence, part 2: the default bench line, rocprofv3 kernel trace + PMC passes of the
# bench command (one counter group per pass)
set -o pipefail
O=gpurun_out/round
mkdir -p $O/prof
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$R"
ARGS="--steps 1 --warmup 1 --no-cpu-baseline"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof/kt -o run --output-format csv -- python3 bench.py $ARGS > $O/prof/kt.log 2>&1 || exit 1
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD" \
           "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --pmc $grp -d $O/prof/pmc$i -o run --output-format csv -- python3 bench.py $ARGS > $O/prof/pmc$i.log 2>&1 || exit 1
done
