#!/bin/bash
# Split round-trip halves: parity tests, then the bench's captured two-stream pipeline
# against per-step graphs round-robin and one step at a time, at the driver's 20 steps and
# at 200.  Results: gpurun_out/bench_modes.jsonl.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_roundtrip.py -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread -rf -k "split or in_flight or graph" > gpurun_out/pytest_pipe.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_pipe.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; exit $rc; fi
STEPS=20 ROUNDS=2 VARIANTS="pipe3:--inflight=3,--pipeline=1,--warmup=5 pipe2:--inflight=2,--pipeline=1,--warmup=5 rr3:--inflight=3,--pipeline=0,--warmup=5 d1:--inflight=1,--warmup=5" \
  bash scripts/gpu_bench_modes.sh || exit $?
cp gpurun_out/bench_modes.jsonl gpurun_out/bench_modes_20.jsonl
STEPS=200 ROUNDS=1 VARIANTS="pipe3:--inflight=3,--pipeline=1,--warmup=5 rr3:--inflight=3,--pipeline=0,--warmup=5 d1:--inflight=1,--warmup=5" \
  bash scripts/gpu_bench_modes.sh || exit $?
cp gpurun_out/bench_modes.jsonl gpurun_out/bench_modes_200.jsonl
