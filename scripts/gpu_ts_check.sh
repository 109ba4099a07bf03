#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_formats.py tests/test_gpu_parity.py tests/test_gpu_sgcht.py -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_fb.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_fb.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/bench_aux.py --only-twostage --reps 20 > gpurun_out/ts.log 2>&1 || exit $?
timeout -k 10 300 python scripts/bench_aux.py --only-twostage --reps 100 > gpurun_out/ts100.log 2>&1 || exit $?
grep stream gpurun_out/ts100.log
grep stream gpurun_out/ts.log
