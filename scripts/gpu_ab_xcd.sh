#!/bin/bash
# A/B of the XCD-aware synthesis workgroup order on C2 (bench) and C3 (bench_aux).
set -u
mkdir -p gpurun_out
for x in 1 0; do
  PFB_SYNTH_XCD=$x timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab_xcd$x.json 2>/dev/null || exit $?
  PFB_SYNTH_XCD=$x timeout -k 10 200 python scripts/bench_aux.py --reps 3 > gpurun_out/ab_aux_xcd$x.jsonl 2>/dev/null || exit $?
  echo "xcd=$x"; python -c "import json;d=json.load(open('gpurun_out/ab_xcd$x.json'));print(d['value'],d['kernels']['synth_block']['avg_ms'])"; grep -E "C3|C2'" gpurun_out/ab_aux_xcd$x.jsonl
done
