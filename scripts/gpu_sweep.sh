#!/bin/bash
# Parameter sweep of the bench (no profiler).  Each run under its own time limit.
set -u
mkdir -p gpurun_out
OUT=gpurun_out/sweep.jsonl
: > $OUT
run() {  # env-prefix args...
  local tag="$1"; shift
  timeout -k 10 180 env "$@" --no-cpu-baseline > gpurun_out/sweep_one.json 2> gpurun_out/sweep_one.err
  local rc=$?
  if [ $rc -ne 0 ]; then echo "FAIL $tag rc=$rc"; tail -5 gpurun_out/sweep_one.err; exit $rc; fi
  python3 -c "import json,sys; d=json.load(open('gpurun_out/sweep_one.json')); k=d['kernels']; print(json.dumps({'tag':'$tag','value':d['value'],'ms':d['ms_per_step'],'kern':{n:round(v['ms_per_step']*1e3,1) for n,v in k.items()}}))" | tee -a $OUT
}
for cmd in "$@"; do
  eval "run $cmd"
done
