# Round-end evidence on one MI355X: smoke + the whole -m gpu suite, the C3 bench line with its
# kernel trace and PMC passes, and the 8-way C4 shares
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/gpu/check.sh || exit 1
bash tools/gpu/profile.sh c3 || exit 1
bash tools/gpu/shares.sh c3 8 3 || exit 1
