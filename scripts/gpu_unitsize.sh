#!/bin/bash
# C2 pipeline throughput vs unit size (Infinity-Cache residency of the stage-1 rows between
# a unit's analysis and its synthesis): bench.py with --n-dat 2^24 / 2^23 / 2^22, D = 3 / 4.
set -u
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
: > gpurun_out/unitsize.jsonl
for rnd in 1 2; do
for n in 16777216 8388608 4194304; do
  for d in 3 4; do
    st=$((20 * 16777216 / n))
    timeout -k 10 200 python bench.py --steps $st --warmup 3 --no-cpu-baseline --n-dat $n --inflight $d \
        --kernel-events 0 >> gpurun_out/unitsize.jsonl 2>> gpurun_out/unitsize.err || exit $?
  done
done
done
python3 -c "
import json
for l in open('gpurun_out/unitsize.jsonl'):
    d=json.loads(l); c=d['config']; print(c['n_dat_per_unit'], c['steps_in_flight'], d['steps'], round(d['value']), d['ms_per_step'])
"
