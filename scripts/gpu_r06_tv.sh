#!/bin/bash
# Round 6: where the C2 streaming analysis spends its time — compile-time timing variants
# (PFB_ANA_TV: 1 no FIR, 2 no FFT, 4 no window slide; results invalid) with and without the
# memory masks (PFB_TIMING_MASK=7: no input loads, no stores reach memory), experiments build.
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
ROUNDS=2 timeout -k 10 900 bash scripts/gpu_ab.sh tv0:PFB_ANA_TV=0 tv1:PFB_ANA_TV=1 tv2:PFB_ANA_TV=2 tv3:PFB_ANA_TV=3 \
    tv4:PFB_ANA_TV=4 tv7:PFB_ANA_TV=7 tv0m7:PFB_ANA_TV=0,PFB_TIMING_MASK=7 tv1m7:PFB_ANA_TV=1,PFB_TIMING_MASK=7 \
    tv2m7:PFB_ANA_TV=2,PFB_TIMING_MASK=7 tv3m7:PFB_ANA_TV=3,PFB_TIMING_MASK=7 tv7m7:PFB_ANA_TV=7,PFB_TIMING_MASK=7 \
    > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 4; }
cp gpurun_out/ab.jsonl gpurun_out/tv_ab.jsonl
python3 - <<'PY'
import json
for l in open("gpurun_out/tv_ab.jsonl"):
    d = json.loads(l); print(d["tag"], {k: v["us"] for k, v in d.items() if isinstance(v, dict) and "us" in v})
PY
