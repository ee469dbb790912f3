# Round-5 measurements of the new paths (one box, one call):
#   the C3 bench line; the reference's redraw (--rebuild) with the walk structures built on the
#   device and on the host; the reference-walk mode (inw_wide_walk=0) with and without the
#   stackless walks; C5 with one WRITE_SIZE PMC pass (nontemporal framebuffer stores); C2 with the
#   LDS bank-conflict counters of k_iow03sL.
#   gpurun -- 'bash tools/gpu/r05_measure.sh'
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_measure; rm -rf $O; mkdir -p $O
B="timeout -k 10 300 python3 bench.py --no-cpu-baseline"
$B --steps 5 > $O/c3.json 2> $O/c3.err || exit 1
$B --steps 5 --rebuild > $O/c3_rebuild_dev.json 2> $O/c3_rebuild_dev.err || exit 1
$B --steps 5 --rebuild --opt inw_device_build=0 > $O/c3_rebuild_host.json 2> $O/c3_rebuild_host.err || exit 1
$B --steps 2 --spp 64 --opt inw_wide_walk=0 --opt inw_stackless=1 > $O/c3_ref_sl.json 2> $O/c3_ref_sl.err || exit 1
$B --steps 2 --spp 64 --opt inw_wide_walk=0 --opt inw_stackless=0 > $O/c3_ref_stack.json 2> $O/c3_ref_stack.err || exit 1
$B --steps 2 --spp 64 --opt inw_wide_walk=0 --opt inw_stackless=1 --opt inw_order=2 > $O/c3_ref_sl_sm.json 2> $O/c3_ref_sl_sm.err || exit 1
$B --steps 2 --spp 64 --opt inw_wide_walk=0 --opt inw_stackless=0 --opt inw_order=2 > $O/c3_ref_stack_sm.json 2> $O/c3_ref_stack_sm.err || exit 1
$B --config c5 --steps 2 > $O/c5.json 2> $O/c5.err || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_c5w -o run --output-format csv -- python3 bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline > $O/pmc_c5w.log 2>&1 || exit 1
$B --config c2 --steps 3 > $O/c2.json 2> $O/c2.err || exit 1
timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS -d $O/pmc_c2lds -o run --output-format csv -- python3 bench.py --config c2 --steps 1 --warmup 1 --no-cpu-baseline > $O/pmc_c2lds.log 2>&1 || exit 1
echo done
