#!/bin/bash
# Kernel trace of the two-stage cascade's stream call (carry read in the analysis window
# prologue: one analysis launch + one carry copy per stage).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/tsprof2 -o run \
    -- python3 $GRAFT_REPO_ROOT/scripts/bench_aux.py --only-twostage > $GRAFT_REPO_ROOT/gpurun_out/tsprof2.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/tsprof2.log
exit $rc
