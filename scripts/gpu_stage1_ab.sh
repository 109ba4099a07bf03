#!/bin/bash
# Stage-1 rows A/B (stored vs recomputed): the bit-identity tests, then interleaved bench
# runs of both modes (the driver's 20-step command) and kernel traces of each.
set -u
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_roundtrip.py -k "recomputed or split or close" -x -q \
    -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/stage1_tests.log 2>&1
rc=$?; tail -5 gpurun_out/stage1_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
: > gpurun_out/stage1_ab.jsonl
for round in 1 2; do
  for m in stored recomputed; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --stage1 $m >> gpurun_out/stage1_ab.jsonl 2> gpurun_out/stage1_ab.err || exit $?
  done
done
python3 -c "
import json
for l in open('gpurun_out/stage1_ab.jsonl'):
    d=json.loads(l); print(d['config']['stage1_rows'], d['value'], d['ms_per_step'], d['ms_per_step_serial'], {k:round(v['avg_ms']*1e3,1) for k,v in d['kernels'].items()})
"
cd /tmp
for m in stored recomputed; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$m -o run \
      -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --inflight 1 --stage1 $m > $R/gpurun_out/prof_$m.log 2>&1 || exit $?
  grep -E "analysis_stream|synth_wave" $R/gpurun_out/prof_$m/run_kernel_stats.csv | cut -d, -f1-4
done
