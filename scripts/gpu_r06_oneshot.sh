#!/bin/bash
# Round 6: shorter-lived workgroups for the two persistent streaming kernels (the copy probe:
# a one-shot grid copies at 6.3-6.6 TB/s, persistent loops at 4.7-5.5) — the C2 streaming
# analysis with S steps per workgroup (PFB_ANA_STEPS) and the C3 FIR with more, shorter
# ranges (PFB_FIR_LDS_WGS workgroups), experiments build.
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd $R
ROUNDS=2 timeout -k 10 900 bash scripts/gpu_ab.sh s0 s1:PFB_ANA_STEPS=1 s2:PFB_ANA_STEPS=2 s3:PFB_ANA_STEPS=3 \
    s5:PFB_ANA_STEPS=5 > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 4; }
cp gpurun_out/ab.jsonl gpurun_out/anasteps_ab.jsonl
python3 - <<'PY'
import json
for l in open("gpurun_out/anasteps_ab.jsonl"):
    d = json.loads(l); print(d["tag"], {k: v["us"] for k, v in d.items() if isinstance(v, dict) and "us" in v})
PY
ROUNDS=2 timeout -k 10 900 bash scripts/gpu_c3_kernel_ab.sh w2k w4k:PFB_FIR_LDS_WGS=4096 w8k:PFB_FIR_LDS_WGS=8192 \
    w16k:PFB_FIR_LDS_WGS=16384 w32k:PFB_FIR_LDS_WGS=32768 > gpurun_out/c3k.log 2>&1 || { tail -5 gpurun_out/c3k.log; exit 5; }
cp gpurun_out/c3k.log gpurun_out/firwgs_ab.log
grep -A1 "==" gpurun_out/firwgs_ab.log | grep -v "^--" ; grep "fir_lds" gpurun_out/firwgs_ab.log
