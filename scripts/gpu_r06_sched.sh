#!/bin/bash
# Round 6: workgroup-order / range-count A/B of the C2 (ab_kernels.py) and C3 (per-kernel
# rocprof stats) kernels, experiments build.  C2V / C3V: variant lists ("tag:ENV=V,ENV=V").
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
if [ -n "${C2V:-}" ]; then
  ROUNDS=${ROUNDS:-2} timeout -k 10 900 bash scripts/gpu_ab.sh $C2V > gpurun_out/ab_sched.log 2>&1 || { tail -5 gpurun_out/ab_sched.log; exit 1; }
  python3 - <<'PY'
import json
for l in open("gpurun_out/ab.jsonl"):
    d = json.loads(l)
    print(f'{d["tag"]:14s}', " ".join(f'{k}={v["us"]:.1f}' for k, v in d.items() if isinstance(v, dict) and "us" in v))
PY
fi
if [ -n "${C3V:-}" ]; then
  ROUNDS=${ROUNDS:-2} timeout -k 10 900 bash scripts/gpu_c3_kernel_ab.sh $C3V > gpurun_out/c3k.log 2>&1 || { tail -5 gpurun_out/c3k.log; exit 1; }
  cat gpurun_out/c3k.log
fi
