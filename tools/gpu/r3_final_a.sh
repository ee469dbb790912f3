# round-3 evidence for the C3 headline: profile (bench line + kernel trace + PMC), 8-way shares,
# multi-rank rehearsal
set -o pipefail
bash tools/gpu/profile.sh c3 || exit 1
bash tools/gpu/shares.sh c3 8 || exit 1
bash tools/gpu/multirank.sh c3 || exit 1
