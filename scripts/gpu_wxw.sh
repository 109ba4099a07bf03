#!/bin/bash
# C2 wave synthesis with cross-wave pass-1 loads (experiments build, PFB_WAVE_XW=1): the C2 /
# C4 round-trip parity tests through it, then per-kernel A/B and in-flight A/B.
set -u
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
EXP=$R/ska-pst-dsp-model_amd/lib/libpfb_hip_exp.so
PFB_HIP_LIB=$EXP PFB_WAVE_XW=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_roundtrip.py -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread -rf -k "c2 or c4 or roundtrip_matches or fused or in_flight" > gpurun_out/pytest_wxw.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_wxw.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; exit $rc; fi
ROUNDS=3 bash scripts/gpu_ab.sh base xw:PFB_WAVE_XW=1 > /dev/null || exit $?
cat gpurun_out/ab.jsonl
ROUNDS=2 VARIANTS="exp xw:PFB_WAVE_XW=1" bash scripts/gpu_inflight_ab.sh || exit $?
