#!/bin/bash
# C3 round-trip A/B of experiments-build variants: digests (bit-identity) then ROUNDS
# interleaved timings of scripts/bench_aux.py --only-mid.  Each argument is "tag" or
# "tag:ENV=VAL,ENV2=VAL".  Results: gpurun_out/c3_ab.jsonl, gpurun_out/c3_digest.jsonl.
set -u
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
EXP=$R/ska-pst-dsp-model_amd/lib/libpfb_hip_exp.so
: > gpurun_out/c3_ab.jsonl
: > gpurun_out/c3_digest.jsonl
for v in "$@"; do
  tag=${v%%:*}; envs=""
  if [ "$tag" != "$v" ]; then envs=${v#*:}; envs=${envs//,/ }; fi
  env PFB_HIP_LIB=$EXP $envs timeout -k 10 120 python scripts/rt_digest.py --workload ${WL:-c3} --tag "$tag" \
      >> gpurun_out/c3_digest.jsonl 2> gpurun_out/c3_ab.err
  rc=$?; if [ $rc -ne 0 ]; then echo "digest $tag rc=$rc"; tail -5 gpurun_out/c3_ab.err; exit $rc; fi
done
cat gpurun_out/c3_digest.jsonl
for round in $(seq 1 ${ROUNDS:-2}); do
  for v in "$@"; do
    tag=${v%%:*}; envs=""
    if [ "$tag" != "$v" ]; then envs=${v#*:}; envs=${envs//,/ }; fi
    env PFB_HIP_LIB=$EXP $envs timeout -k 10 120 python scripts/bench_aux.py --only-mid --reps ${REPS:-10} \
        | sed "s/^{/{\"tag\": \"$tag\", /" >> gpurun_out/c3_ab.jsonl 2> gpurun_out/c3_ab.err
    rc=$?; if [ $rc -ne 0 ]; then echo "variant $tag rc=$rc"; tail -5 gpurun_out/c3_ab.err; exit $rc; fi
  done
done
cat gpurun_out/c3_ab.jsonl
