#!/bin/bash
# Stream objects with the one-launch stitch + carry copy: the stream / two-stage / sgcht
# parity tests, then the two-stage cascade interleaved with the previous library.
set -u
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -rf \
    -k "stream or carry or two_stage or twostage or sgcht or filterbank or cascade" > gpurun_out/pytest_carry.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_carry.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; exit $rc; fi
: > gpurun_out/ts_ab.jsonl
for round in 1 2 3; do
  for v in new prev; do
    lib=$R/ska-pst-dsp-model_amd/lib/libpfb_hip.so; [ $v = prev ] && lib=$R/ska-pst-dsp-model_amd/lib/libpfb_hip_prev.so
    PFB_HIP_LIB=$lib timeout -k 10 200 python scripts/bench_aux.py --only-twostage > gpurun_out/ts.jsonl 2> gpurun_out/ts.err || { tail -3 gpurun_out/ts.err; exit 1; }
    python3 -c "
import json
for l in open('gpurun_out/ts.jsonl'):
    d=json.loads(l)
    if 'stream call' in d['kernel']: print(json.dumps({'tag': '$v', 'ms': d['ms']}))" | tee -a gpurun_out/ts_ab.jsonl
  done
done
