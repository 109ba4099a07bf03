#!/bin/bash
# Round 6: co-residency A/B of the two-stream pipelines (experiments build).  C2: bench.py's
# captured pipeline (inflight_ab.py --pipeline 1, 3 units in flight) under launch-geometry
# knobs (analysis / synthesis workgroups per CU); C3: scripts/gpu_r06_c3pipe.sh.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
EXP=$GRAFT_REPO_ROOT/ska-pst-dsp-model_amd/lib/libpfb_hip_exp.so
C2V=${C2VARIANTS:-base a1:PFB_ANA_WG_PER_CU=1 w2:PFB_WAVE_PER_CU=2 a1w2:PFB_ANA_WG_PER_CU=1,PFB_WAVE_PER_CU=2 w1:PFB_WAVE_PER_CU=1}
: > gpurun_out/c2pipe.jsonl
for round in $(seq 1 ${ROUNDS:-2}); do
  for v in $C2V; do
    tag=${v%%:*}; envs=""
    if [ "$tag" != "$v" ]; then envs=${v#*:}; envs=${envs//,/ }; fi
    env PFB_HIP_LIB=$EXP $envs timeout -k 10 150 python scripts/inflight_ab.py --tag $tag --inflight 3 --pipeline 1 --steps 20 --reps 5 \
        >> gpurun_out/c2pipe.jsonl 2> gpurun_out/c2pipe.err || { rc=$?; tail -5 gpurun_out/c2pipe.err; exit $rc; }
  done
done
cat gpurun_out/c2pipe.jsonl
if [ -n "${C3:-1}" ]; then bash scripts/gpu_r06_c3pipe.sh || exit $?; fi
