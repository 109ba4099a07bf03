#!/bin/bash
# In-flight steps on one GPU: bench.py --inflight D for C2 and C4, the C3 round trip with D
# units in flight (bench_aux.py --only-mid --inflight D), and a kernel trace of the D = 3
# C2 bench (overlapping dispatches).  Stops at the first failing GPU step.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
VARIANTS="g1d1:--graph=1,--inflight=1 g1d2:--graph=1,--inflight=2 g1d3:--graph=1,--inflight=3 g1d4:--graph=1,--inflight=4" \
  ROUNDS=2 bash scripts/gpu_bench_modes.sh || exit $?
cp gpurun_out/bench_modes.jsonl gpurun_out/bench_modes_c2.jsonl
VARIANTS="c4d1:--graph=1,--inflight=1 c4d3:--graph=1,--inflight=3" BENCH_ARGS="--workload c4" \
  ROUNDS=2 STEPS=20 bash scripts/gpu_bench_modes.sh || exit $?
cp gpurun_out/bench_modes.jsonl gpurun_out/bench_modes_c4.jsonl
: > gpurun_out/c3_inflight.jsonl
for d in 1 2 3 1 2 3; do
  timeout -k 10 240 python scripts/bench_aux.py --only-mid --inflight $d >> gpurun_out/c3_inflight.jsonl 2> gpurun_out/c3.err
  rc=$?; if [ $rc -ne 0 ]; then echo "c3 inflight $d rc=$rc"; tail -5 gpurun_out/c3.err; exit $rc; fi
done
cat gpurun_out/c3_inflight.jsonl
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_d3 -o run \
    -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --kernel-events 0 --inflight 3 > $R/gpurun_out/prof_d3.log 2>&1
rc=$?; cd $R
if [ $rc -ne 0 ]; then echo "rocprof rc=$rc"; tail -5 gpurun_out/prof_d3.log; exit $rc; fi
echo done
