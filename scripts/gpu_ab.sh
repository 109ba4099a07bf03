#!/bin/bash
# A/B of kernel variants in one GPU session (experiments build).  Each argument is a variant
# "tag" or "tag:ENV=VAL,ENV2=VAL"; each runs scripts/ab_kernels.py in its own process and
# ROUNDS rounds interleave the variants.  Results: gpurun_out/ab.jsonl.
#   bash scripts/gpu_ab.sh new old:PFB_SYNTH_WAVE=0
set -u
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
EXP=$R/ska-pst-dsp-model_amd/lib/libpfb_hip_exp.so
: > gpurun_out/ab.jsonl
for round in $(seq 1 ${ROUNDS:-2}); do
  for v in "$@"; do
    tag=${v%%:*}; envs=""
    if [ "$tag" != "$v" ]; then envs=${v#*:}; envs=${envs//,/ }; fi
    env PFB_HIP_LIB=$EXP $envs timeout -k 10 120 python scripts/ab_kernels.py --tag "$tag" ${AB_ARGS:-} \
        >> gpurun_out/ab.jsonl 2> gpurun_out/ab.err
    rc=$?; if [ $rc -ne 0 ]; then echo "variant $tag rc=$rc"; tail -5 gpurun_out/ab.err; exit $rc; fi
  done
done
cat gpurun_out/ab.jsonl
