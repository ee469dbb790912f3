# PMC of a lone wave (one pixel, sequential kernel, wave-cooperative closest hits)
set -o pipefail
O=gpurun_out/lone
rm -rf $O && mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd "$R"
# (tools/lone_pixel.py runs the sequential kernel with cooperative closest hits: rt_options
# iow_spec = 0, iow_coop_max = 4)
timeout -k 10 120 python3 tools/lone_pixel.py > $O/run.json 2> $O/run.err || exit 1
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_SMEM" \
           "SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d $O/pmc$i -o run --output-format csv -- python3 tools/lone_pixel.py > $O/pmc$i.log 2>&1 || exit 1
done
