#!/bin/bash
# How the C2 bench value depends on the timed region's length and the warm-up count
# (driver: --steps 20 --warmup 5).  Results: gpurun_out/warm.jsonl.
set -u
mkdir -p gpurun_out
: > gpurun_out/warm.jsonl
for v in "20 5" "20 20" "60 5" "200 5" "20 5"; do
  set -- $v
  timeout -k 10 180 python bench.py --steps $1 --warmup $2 --no-cpu-baseline --kernel-events 0 > gpurun_out/w.json 2> gpurun_out/w.err || { tail -3 gpurun_out/w.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/w.json')); print(json.dumps({'steps': $1, 'warmup': $2, 'value': d['value'], 'ms_per_step': d['ms_per_step']}))" | tee -a gpurun_out/warm.jsonl
done
