#!/bin/bash
# Launch-mode A/B of the headline bench on one GPU: HIP graph vs plain launches, and D steps
# in flight (bench.py --inflight D).  Each variant is its own bench process (release library);
# ROUNDS rounds interleave the variants.  Results: gpurun_out/bench_modes.jsonl.
set -u
mkdir -p gpurun_out
: > gpurun_out/bench_modes.jsonl
VARIANTS=${VARIANTS:-"g1d1:--graph=1,--inflight=1 g0d1:--graph=0,--inflight=1 g1d2:--graph=1,--inflight=2 g0d2:--graph=0,--inflight=2"}
for round in $(seq 1 ${ROUNDS:-2}); do
  for v in $VARIANTS; do
    tag=${v%%:*}; a=${v#*:}; a=${a//,/ }
    timeout -k 10 180 python bench.py --steps ${STEPS:-40} --warmup 3 --no-cpu-baseline --kernel-events 0 $a ${BENCH_ARGS:-} \
        > gpurun_out/bm.json 2> gpurun_out/bm.err
    rc=$?; if [ $rc -ne 0 ]; then echo "variant $tag rc=$rc"; tail -5 gpurun_out/bm.err; exit $rc; fi
    python3 -c "
import json,sys; d=json.load(open('gpurun_out/bm.json'))
print(json.dumps({'tag': '$tag', 'args': '$a ${BENCH_ARGS:-}', 'value': d['value'], 'ms_per_step': d['ms_per_step']}))" \
        | tee -a gpurun_out/bench_modes.jsonl
  done
done
