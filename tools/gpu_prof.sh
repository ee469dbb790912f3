# rocprofv3 passes over a short bench run: kernel trace + stats, then PMC groups one by one
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
ARGS=${PROF_ARGS:---spp 2 --width 600 --height 400 --steps 1 --warmup 0 --no-cpu-baseline}
rocprofv3 -L > gpurun_out/prof/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/kt -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof/kt.log 2>&1 || exit 1
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d gpurun_out/prof/pmc$i -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/prof/pmc$i.log 2>&1 || echo "pmc group $i failed" >> gpurun_out/prof/errors.txt
done
