# Round-4 profiles of the secondary configs: C5 (k_inw_sm<true,...>) and C2 (k_iow03sL), each a
# bench line, a kernel trace and the PMC passes of tools/gpu/profile.sh (STEPS frames for the line).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for cfg in ${CFGS:-c5 c2}; do
  STEPS=${STEPS:-2} timeout -k 10 1000 bash tools/gpu/profile.sh $cfg > gpurun_out/prof_$cfg.txt 2>&1 || { echo PROFILE_${cfg}_FAILED; exit 1; }
done
