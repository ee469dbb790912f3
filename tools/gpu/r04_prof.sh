# Round-4 profiles: C3 (the bench config), C5 (k_inw_sm<true,...>) and C2 (k_iow03sL): a bench
# line, a kernel trace and the PMC passes of tools/gpu/profile.sh each.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for cfg in ${CFGS:-c3 c5 c2}; do
  S=10; [ $cfg != c3 ] && S=2
  STEPS=$S timeout -k 10 1200 bash tools/gpu/profile.sh $cfg > gpurun_out/prof_$cfg.txt 2>&1 || { echo PROFILE_${cfg}_FAILED; exit 1; }
done
