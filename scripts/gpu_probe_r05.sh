#!/bin/bash
# Round-5 probes: HBM streaming ceilings (copy / read / write) and a kernel-trace profile
# of the TwoStage cascade stream call.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python scripts/hbm_probe.py > gpurun_out/hbm_probe.jsonl 2> gpurun_out/hbm_probe.err || exit $?
cat gpurun_out/hbm_probe.jsonl
rm -rf gpurun_out/prof_ts
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ts -o ts -- \
    python scripts/bench_aux.py --only-twostage --reps 20 > gpurun_out/ts.log 2>&1 || exit $?
cat gpurun_out/ts.log | tail -3
f=$(find gpurun_out/prof_ts -name "*kernel_stats.csv" | head -1); cut -d, -f1-5 "$f" | head -15
