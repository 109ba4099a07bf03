#!/bin/bash
# Round 6: is the C2 analysis' FFT share its arithmetic or its channelised-row stores
# (PFB_ANA_TV=16: FFT computed, stores not issued; results invalid), and the two-stream
# pipeline's co-residency under launch-geometry knobs (inflight_ab.py --pipeline 1).
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
ROUNDS=3 timeout -k 10 600 bash scripts/gpu_ab.sh tv0:PFB_ANA_TV=0 tv16:PFB_ANA_TV=16 tv2:PFB_ANA_TV=2 \
    > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 4; }
cp gpurun_out/ab.jsonl gpurun_out/store_ab.jsonl
python3 - <<'PY'
import json
for l in open("gpurun_out/store_ab.jsonl"):
    d = json.loads(l); print(d["tag"], {k: v["us"] for k, v in d.items() if isinstance(v, dict) and "us" in v})
PY
C3=  ROUNDS=2 C2VARIANTS="base w1:PFB_WAVE_PER_CU=1 w2:PFB_WAVE_PER_CU=2 a1:PFB_ANA_WG_PER_CU=1 a3w:PFB_ANA_WPE=3,PFB_ANA_WG_PER_CU=2 a3w3:PFB_ANA_WPE=3" \
    timeout -k 10 900 bash scripts/gpu_r06_coresid.sh > gpurun_out/coresid.log 2>&1 || { tail -5 gpurun_out/coresid.log; exit 5; }
cat gpurun_out/c2pipe.jsonl
