# Round-6 final checks: the whole GPU suite, smoke(), and the C2 profile (octant cull).
#   gpurun -- 'bash tools/gpu/r06_final.sh [suite|c2|ns]'
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_final; mkdir -p $O
case ${1:-suite} in
  suite) timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_suite.log 2>&1 || { tail -40 $O/gpu_suite.log; exit 1; }
         tail -3 $O/gpu_suite.log
         timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
         tail -3 $O/smoke.log ;;
  c2) STEPS=3 bash tools/gpu/profile.sh c2 || exit 1 ;;
  ns) STEPS=1 bash tools/gpu/profile.sh ns || exit 1 ;;
esac
echo done
