#!/bin/bash
# SKA-Mid wave synthesis, second version: parity subset on the release build (cross-wave
# pass-1 loads) and on the experiments build with PFB_W5_XW=0, then C3 round-trip A/B.
set -u
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
EXP=$R/ska-pst-dsp-model_amd/lib/libpfb_hip_exp.so
PFB_PARITY_LOG=$R/gpurun_out/parity_w5.jsonl timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread -rf -k "nf512 or c3 or 4096 or baseline_shapes or roundtrip_matches or mid" \
    > gpurun_out/pytest_w5.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_w5.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; exit $rc; fi
PFB_HIP_LIB=$EXP PFB_W5_XW=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread -rf -k "nf512" > gpurun_out/pytest_w5_xw0.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_w5_xw0.log
if [ $rc -ne 0 ]; then echo "pytest xw0 rc=$rc"; exit $rc; fi
: > gpurun_out/c3_masks.jsonl
for round in 1 2; do
  for v in rel exp xw0:PFB_W5_XW=0 block:PFB_SYNTH_WAVE512=0 mask_z:PFB_TIMING_MASK=1 mask_all:PFB_TIMING_MASK=3; do
    tag=${v%%:*}; envs=""
    if [ "$tag" != "$v" ]; then envs=${v#*:}; envs=${envs//,/ }; fi
    lib=$EXP; [ "$tag" = "rel" ] && lib=$R/ska-pst-dsp-model_amd/lib/libpfb_hip.so
    env PFB_HIP_LIB=$lib $envs timeout -k 10 200 python scripts/bench_aux.py --only-mid > gpurun_out/c3m.json 2> gpurun_out/c3m.err
    rc=$?; if [ $rc -ne 0 ]; then echo "variant $tag rc=$rc"; tail -5 gpurun_out/c3m.err; exit $rc; fi
    python3 -c "import json; d=json.load(open('gpurun_out/c3m.json')); print(json.dumps({'tag': '$tag', 'env': '$envs', 'ms': d['ms']}))" | tee -a gpurun_out/c3_masks.jsonl
  done
done
