# North-star workload (IOW-03 final scene, 1920x1080, 500 spp): 8-way shares for heavy-first settings
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/ns_heavy; rm -rf $O; mkdir -p $O
for h in ${HEAVY:-default 48 96}; do
  if [ "$h" = "default" ]; then X=""; else X="--opt spec_heavy=$h"; fi
  timeout -k 10 900 bash tools/gpu/shares.sh ns 8 1 $X > $O/h_$h.txt 2>&1 || exit 1
  cp gpurun_out/shares_ns_8/summary.json $O/summary_h_$h.json
done
