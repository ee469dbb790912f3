# Round-6 first check of k_inw_pm's GQ instance (quantised nodes + LDS staging + global FStack):
# C3 bench lines with and without it (same box), then the -m gpu suite.
#   gpurun -- 'bash tools/gpu/r06_gq.sh'
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_gq; rm -rf $O; mkdir -p $O
B="timeout -k 10 300 python3 bench.py"
$B --steps 5 > $O/c3_gq.json 2> $O/c3_gq.err || exit 1
$B --steps 5 --no-cpu-baseline --opt inw_qnodes=0 > $O/c3_base.json 2> $O/c3_base.err || exit 1
$B --steps 5 --no-cpu-baseline > $O/c3_gq2.json 2> $O/c3_gq2.err || exit 1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
echo done
