#!/bin/bash
# Round 6: release-build GPU tests (STEPS of gpu_r06.sh, default "tests"), then an interleaved
# A/B of experiments-build variants through gpu_ab.sh (VARIANTS, ROUNDS).  Stops at the first
# failure that is not a test failure.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
STEPS=${STEPS:-tests} bash scripts/gpu_r06.sh || exit $?
if [ -n "${VARIANTS:-}" ]; then
  ROUNDS=${ROUNDS:-2} timeout -k 10 900 bash scripts/gpu_ab.sh $VARIANTS > gpurun_out/ab.log 2>&1 || { rc=$?; tail -20 gpurun_out/ab.log; exit $rc; }
  cat gpurun_out/ab.log
fi
