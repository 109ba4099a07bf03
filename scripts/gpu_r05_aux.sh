#!/bin/bash
# Round-5 auxiliary records: the C4 bench line on one GPU and every bench_aux configuration.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --workload c4 --steps 20 --warmup 3 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || exit $?
tail -c 400 gpurun_out/bench_c4.json
timeout -k 10 900 python scripts/bench_aux.py --reps 10 > gpurun_out/bench_aux.jsonl 2> gpurun_out/bench_aux.err || exit $?
cut -c1-140 gpurun_out/bench_aux.jsonl
