#!/bin/bash
# One GPU session: parity tests (error statistics logged), smoke, bench (C2 headline and
# the C4 unit on one GPU), kernel-trace profile.
# Stops at the first fault/abort/timeout (exit codes other than 0 or 1 from pytest).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-10}
rm -f gpurun_out/parity_errors.jsonl
PFB_PARITY_LOG=$GRAFT_REPO_ROOT/gpurun_out/parity_errors.jsonl timeout -k 10 900 \
    python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps $STEPS --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps $STEPS --warmup 3 --workload c4 --no-cpu-baseline > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err
rc=$?; echo "bench c4 rc=$rc"; cat gpurun_out/bench_c4.json; tail -3 gpurun_out/bench_c4.err
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run \
    -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --inflight 1 > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"
exit $rc
