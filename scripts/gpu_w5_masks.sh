#!/bin/bash
# Where the SKA-Mid wave synthesis spends its time: C3 round trips (experiments build) with
# the synthesis's Z loads and/or output stores dropped (PFB_TIMING_MASK, results invalid),
# and its persistent range count varied.  Results: gpurun_out/c3_masks.jsonl.
set -u
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
EXP=$R/ska-pst-dsp-model_amd/lib/libpfb_hip_exp.so
: > gpurun_out/c3_masks.jsonl
for round in 1 2; do
  for v in base mask_z:PFB_TIMING_MASK=1 mask_st:PFB_TIMING_MASK=2 mask_all:PFB_TIMING_MASK=3 r1:PFB_W5_RANGES=1 r6:PFB_W5_RANGES=6 block:PFB_SYNTH_WAVE512=0; do
    tag=${v%%:*}; envs=""
    if [ "$tag" != "$v" ]; then envs=${v#*:}; envs=${envs//,/ }; fi
    env PFB_HIP_LIB=$EXP $envs timeout -k 10 200 python scripts/bench_aux.py --only-mid > gpurun_out/c3m.json 2> gpurun_out/c3m.err
    rc=$?; if [ $rc -ne 0 ]; then echo "variant $tag rc=$rc"; tail -5 gpurun_out/c3m.err; exit $rc; fi
    python3 -c "import json; d=json.load(open('gpurun_out/c3m.json')); print(json.dumps({'tag': '$tag', 'env': '$envs', 'ms': d['ms']}))" | tee -a gpurun_out/c3_masks.jsonl
  done
done
