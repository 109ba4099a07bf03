#!/bin/bash
# Cache-policy A/B of the C2 round trip: variant libraries built with -DPFB_AUX_*=2 (nt) on
# the analysis input loads, channelised-row stores, stage-1 row stores, synthesis output
# stores (lib/libpfb_hip_<tag>.so, see pfb_common.hpp), interleaved inflight_ab.py runs
# (D = 3, the bench's regime), two rounds; the C3 nontemporal-store variant
# (-DPFB_NT_C3=1, lib/libpfb_hip_c3nt.so) through gpu_c3_ab.sh; then the bandwidth probe.
set -u
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
OUT=gpurun_out/aux_ab.jsonl
: > $OUT
for round in $(seq 1 ${ROUNDS:-2}); do
  for tag in ${TAGS:-base chan2 zst2 out2 in2 co2}; do
    [ "$tag" = base ] && tag=""
    lib=ska-pst-dsp-model_amd/lib/libpfb_hip${tag:+_$tag}.so
    for d in 3; do
      PFB_HIP_LIB=$lib timeout -k 10 120 python scripts/inflight_ab.py --tag "${tag:-base}" --inflight $d \
          --steps 40 --reps 5 >> $OUT 2>> gpurun_out/aux_ab.err || exit $?
    done
  done
done
L=ska-pst-dsp-model_amd/lib
if [ "${C3:-1}" = 1 ]; then
  bash scripts/gpu_c3_ab.sh base:PFB_HIP_LIB=$L/libpfb_hip.so c3nt:PFB_HIP_LIB=$L/libpfb_hip_c3nt.so || exit $?
  timeout -k 10 120 ./scripts/bw_probe > gpurun_out/bw_probe.jsonl 2>&1 || exit $?
fi
python3 - <<'EOF'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/aux_ab.jsonl"):
    r = json.loads(l)
    d[(r["tag"], r["inflight"])].append(r["us_per_step"])
for k in sorted(d):
    print(k, d[k])
EOF
