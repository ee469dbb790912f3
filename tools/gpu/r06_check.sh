# Round-6 check on one MI355X: smoke() and the -m gpu suite, then the C3 bench line (with the CPU
# baseline and its parity block), the C5 and C2 lines, and the multi-rank rehearsal (depth included).
#   gpurun -- 'bash tools/gpu/r06_check.sh'
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu/check.sh || exit 1
O=gpurun_out/r06_check; rm -rf $O; mkdir -p $O
timeout -k 10 300 python3 bench.py --steps 5 > $O/c3.json 2> $O/c3.err || exit 1
timeout -k 10 400 python3 bench.py --config c5 --steps 2 --no-cpu-baseline > $O/c5.json 2> $O/c5.err || exit 1
timeout -k 10 300 python3 bench.py --config c2 --steps 2 --no-cpu-baseline > $O/c2.json 2> $O/c2.err || exit 1
bash tools/gpu/multirank.sh c3 > $O/multirank.log 2>&1 || exit 1
echo done
