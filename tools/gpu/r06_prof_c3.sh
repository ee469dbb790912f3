# Round-6 C3 evidence: the bench line, kernel trace and PMC passes of the product (profiles/pmc_c3.json)
# and of the GQ instance (--opt inw_qnodes=1: global 40-float stacks, quantised nodes staged in LDS).
#   gpurun -- 'bash tools/gpu/r06_prof_c3.sh'
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
STEPS=10 bash tools/gpu/profile.sh c3 || exit 1
STEPS=3 BENCH_ARGS="--opt inw_qnodes=1 --no-cpu-baseline" TAG=c3_gq bash tools/gpu/profile.sh c3 || exit 1
echo done
