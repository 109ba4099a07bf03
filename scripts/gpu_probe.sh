#!/bin/bash
# Development probe: timing-mask A/B of the C2 kernels (experiments build) and PMC passes
# over a short C2 bench run.  Stops at the first failing GPU step.
set -u
R=$GRAFT_REPO_ROOT
cd $R
ROUNDS=${ROUNDS:-2} bash scripts/gpu_ab.sh ${AB_VARIANTS:-base mask_z:PFB_TIMING_MASK=1 mask_st:PFB_TIMING_MASK=2 mask_all:PFB_TIMING_MASK=3} || exit $?
[ -n "${NO_PMC:-}" ] && exit 0
rm -rf gpurun_out/pmc_*
bash scripts/gpu_pmc.sh ${PMC_SETS:-} || exit $?
for d in gpurun_out/pmc_[0-9]*/; do python3 scripts/pmc_summary.py $d 2>/dev/null | head -30; done
