#!/bin/bash
# Cache-policy A/B of the TwoStage cascade: variant libraries (lib/libpfb_hip_<tag>.so,
# -DPFB_AUX_STRIDED / -DPFB_AUX_COLMAJOR, pfb_common.hpp) through bench_aux.py
# --only-twostage, ROUNDS interleaved rounds.  Results: gpurun_out/twostage_ab.jsonl.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/twostage_ab.jsonl
for round in $(seq 1 ${ROUNDS:-3}); do
  for tag in ${TAGS:-base st2 cm2}; do
    lib=ska-pst-dsp-model_amd/lib/libpfb_hip.so
    [ "$tag" != base ] && lib=ska-pst-dsp-model_amd/lib/libpfb_hip_$tag.so
    PFB_HIP_LIB=$lib timeout -k 10 120 python scripts/bench_aux.py --only-twostage --reps 20 \
        | sed "s/^{/{\"tag\": \"$tag\", /" >> gpurun_out/twostage_ab.jsonl 2>> gpurun_out/twostage_ab.err || exit $?
  done
done
grep "stream call" gpurun_out/twostage_ab.jsonl | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l); print(d['tag'], d['ms'])
"
