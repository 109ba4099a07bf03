#!/bin/bash
# C3 per-stream cache-policy A/B: variant libraries lib/libpfb_hip_<tag>.so (-DPFB_NT_FIRZ /
# _ROW / _W5, pfb_common.hpp) — interleaved bench_aux.py --only-mid timings, then one
# rocprofv3 kernel trace per variant (per-kernel averages).  Results under gpurun_out/.
set -u
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
TAGS=${TAGS:-base firz1 row0 w50}
: > gpurun_out/c3_policy_ab.jsonl
for round in $(seq 1 ${ROUNDS:-2}); do
  for tag in $TAGS; do
    lib=$R/ska-pst-dsp-model_amd/lib/libpfb_hip.so
    [ "$tag" != base ] && lib=$R/ska-pst-dsp-model_amd/lib/libpfb_hip_$tag.so
    PFB_HIP_LIB=$lib timeout -k 10 120 python scripts/bench_aux.py --only-mid --reps 10 \
        | sed "s/^{/{\"tag\": \"$tag\", /" >> gpurun_out/c3_policy_ab.jsonl 2>> gpurun_out/c3_policy_ab.err || exit $?
  done
done
for tag in $TAGS; do
  lib=$R/ska-pst-dsp-model_amd/lib/libpfb_hip.so
  [ "$tag" != base ] && lib=$R/ska-pst-dsp-model_amd/lib/libpfb_hip_$tag.so
  (cd /tmp && PFB_HIP_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $R/gpurun_out/c3pol_$tag -o run -- python3 $R/scripts/bench_aux.py --only-mid --reps 5 \
      > $R/gpurun_out/c3pol_$tag.log 2>&1) || exit $?
done
python3 - <<'PY'
import csv, json
for l in open("gpurun_out/c3_policy_ab.jsonl"):
    d = json.loads(l); print(d["tag"], d["ms"])
import os
for tag in os.environ.get("TAGS", "base firz1 row0 w50").split():
    rows = list(csv.DictReader(open(f"gpurun_out/c3pol_{tag}/run_kernel_stats.csv")))
    print(tag, {r["Name"][5:30]: round(float(r["AverageNs"]) / 1e3, 1) for r in rows if "pfb::" in r["Name"]})
PY
