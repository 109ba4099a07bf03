#!/bin/bash
# Launch-geometry A/B in the in-flight regime (scripts/inflight_ab.py, experiments build for
# the knobs, the release build as the reference), ROUNDS interleaved rounds.
# Results: gpurun_out/inflight_ab.jsonl.  Stops at the first failing GPU step.
set -u
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
EXP=$R/ska-pst-dsp-model_amd/lib/libpfb_hip_exp.so
: > gpurun_out/inflight_ab.jsonl
for round in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VARIANTS:-rel exp}; do
    tag=${v%%:*}; envs=""
    if [ "$tag" != "$v" ]; then envs=${v#*:}; envs=${envs//,/ }; fi
    lib=$EXP; [ "$tag" = "rel" ] && lib=$R/ska-pst-dsp-model_amd/lib/libpfb_hip.so
    env PFB_HIP_LIB=$lib $envs timeout -k 10 120 python scripts/inflight_ab.py --tag "$tag" ${AB_ARGS:-} \
        >> gpurun_out/inflight_ab.jsonl 2> gpurun_out/inflight_ab.err
    rc=$?; if [ $rc -ne 0 ]; then echo "variant $tag rc=$rc"; tail -5 gpurun_out/inflight_ab.err; exit $rc; fi
  done
done
cat gpurun_out/inflight_ab.jsonl
