# PMC passes of the C4 (INW-01 LBVH) bench frame at spp 32 (full resolution): issue / wait mix
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/pmc4 && mkdir -p gpurun_out/pmc4
ARGS="--config c4 --steps 1 --warmup 0 --no-cpu-baseline --spp 32"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD" \
           "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
           "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
           "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $grp -d gpurun_out/pmc4/pmc$i -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc4/pmc$i.log 2>&1 || exit 1
done
