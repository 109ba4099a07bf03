#!/bin/bash
# Round 6: the SKA-Mid synthesis with compile-time lane-pair twiddles (synth_wave512_kernel
# CT) — Nf-512 / C3 GPU tests on the release build, bit-identity of CT 0 / 1 (rt_digest,
# experiments build), per-kernel rocprof A/B of CT 0 / 1, and the C2 analysis timing masks
# (PFB_TIMING_MASK 1 no input loads, 2 no channelised stores, 4 no stage-1 row stores).
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf \
    -k "${K:-c3 or mid or padded or 4096 or nf512 or sharding or round_trip or roundtrip}" > gpurun_out/pytest_ct.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_ct.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
EXP=$R/ska-pst-dsp-model_amd/lib/libpfb_hip_exp.so
for ct in 1 0; do
  PFB_HIP_LIB=$EXP PFB_W5_CT=$ct timeout -k 10 200 python scripts/rt_digest.py --workload c3 --tag ct$ct \
      >> gpurun_out/ct_digest.jsonl 2> gpurun_out/ct_digest.err || { tail -5 gpurun_out/ct_digest.err; exit 3; }
done
cat gpurun_out/ct_digest.jsonl
ROUNDS=2 timeout -k 10 900 bash scripts/gpu_c3_kernel_ab.sh ct1:PFB_W5_CT=1 ct0:PFB_W5_CT=0 > gpurun_out/c3k.log 2>&1 || exit $?
cat gpurun_out/c3k.log
ROUNDS=2 timeout -k 10 900 bash scripts/gpu_ab.sh m0:PFB_TIMING_MASK=0 m1:PFB_TIMING_MASK=1 m2:PFB_TIMING_MASK=2 \
    m4:PFB_TIMING_MASK=4 m6:PFB_TIMING_MASK=6 m7:PFB_TIMING_MASK=7 > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 4; }
cp gpurun_out/ab.jsonl gpurun_out/ana_masks.jsonl
python3 - <<'PY'
import json
for l in open("gpurun_out/ana_masks.jsonl"):
    d = json.loads(l); print(d["tag"], {k: v["us"] for k, v in d.items() if isinstance(v, dict) and "us" in v})
PY
