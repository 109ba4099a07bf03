#!/bin/bash
# Stream objects reading the carry through a second descriptor in the first window: the
# stream / two-stage / sgcht parity tests, the two-stage cascade and the C2 bench line
# interleaved with the previous library, then the round validation (scripts/gpu_round.sh).
set -u
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -rf \
    -k "stream or carry or two_stage or twostage or sgcht or filterbank or cascade" > gpurun_out/pytest_carry.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_carry.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; exit $rc; fi
: > gpurun_out/ts_ab.jsonl
: > gpurun_out/c2_ab.jsonl
for round in 1 2 3; do
  for v in new prev; do
    lib=$R/ska-pst-dsp-model_amd/lib/libpfb_hip.so; [ $v = prev ] && lib=$R/ska-pst-dsp-model_amd/lib/libpfb_hip_prev.so
    PFB_HIP_LIB=$lib timeout -k 10 200 python scripts/bench_aux.py --only-twostage > gpurun_out/ts.jsonl 2> gpurun_out/ts.err || { tail -3 gpurun_out/ts.err; exit 1; }
    python3 -c "
import json
for l in open('gpurun_out/ts.jsonl'):
    d=json.loads(l)
    if 'stream call' in d['kernel']: print(json.dumps({'tag': '$v', 'ms': d['ms']}))" | tee -a gpurun_out/ts_ab.jsonl
    # bench.py refuses PFB_HIP_LIB: swap the release file in place instead
    L=$R/ska-pst-dsp-model_amd/lib
    [ $v = prev ] && { cp $L/libpfb_hip.so $L/libpfb_hip_new.so && cp $L/libpfb_hip_prev.so $L/libpfb_hip.so; }
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/c2.json 2> gpurun_out/c2.err
    brc=$?
    [ $v = prev ] && mv $L/libpfb_hip_new.so $L/libpfb_hip.so
    [ $brc -ne 0 ] && { tail -3 gpurun_out/c2.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('gpurun_out/c2.json').read().strip().splitlines()[-1])
print(json.dumps({'tag': '$v', 'value': d['value'], 'ms': d['ms_per_step'], 'kernels': {k: v.get('avg_ms') for k, v in d.get('kernels', {}).items()} if isinstance(d.get('kernels'), dict) else None}))" | tee -a gpurun_out/c2_ab.jsonl
  done
done
rm -f $R/ska-pst-dsp-model_amd/lib/libpfb_hip_prev.so
STEPS=20 bash scripts/gpu_round.sh
