# Round 3 baseline: C3 (INW-01 LBVH, 1920x1080, 500 spp) kernel trace + PMC of the round-2 kernels,
# and the per-pixel kernel (RT_INW_SPEC=0) for comparison
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd "$R"
O=gpurun_out/r3a
rm -rf $O && mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_c3_kt.log 2>&1 || exit 1
RT_INW_SPEC=0 timeout -k 10 240 python3 bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_c3_pixel.log 2>&1 || exit 1
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d $O/pmc$i -o run --output-format csv -- python3 bench.py --config c4 --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc$i.log 2>&1 || exit 1
done
