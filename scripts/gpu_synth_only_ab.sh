#!/bin/bash
# Interleaved A/B of the standalone C2 synthesis over experiments-build knobs
# ("tag:ENV=V[,ENV=V]" or "tag:LIB=variant" for lib/libpfb_hip_<variant>.so), ROUNDS rounds.  Results: gpurun_out/synth_only_ab.jsonl.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/synth_only_ab.jsonl
for round in $(seq 1 ${ROUNDS:-3}); do
  for spec in "$@"; do
    tag=${spec%%:*}; envs=${spec#*:}; [ "$envs" = "$spec" ] && envs=""
    lib=ska-pst-dsp-model_amd/lib/libpfb_hip_exp.so
    case "$envs" in LIB=*) lib=ska-pst-dsp-model_amd/lib/libpfb_hip_${envs#LIB=}.so; envs="";; esac
    env $(echo "$envs" | tr ',' ' ') PFB_HIP_LIB=$lib \
      timeout -k 10 120 python scripts/synth_only_time.py --tag $tag >> gpurun_out/synth_only_ab.jsonl \
      2>> gpurun_out/synth_only_ab.err || exit $?
  done
done
cat gpurun_out/synth_only_ab.jsonl
