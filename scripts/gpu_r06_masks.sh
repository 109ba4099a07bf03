#!/bin/bash
# Round 6: timing decomposition of the two wave synthesis kernels (experiments build; results
# invalid under a mask).  PFB_TIMING_MASK bits: 1 no Z loads, 2 no output stores.
# Compile-time timing variants: C2 PFB_WAVE_V=9/17/25 (V 1 + 8 wave barriers instead of the
# block loop's workgroup barriers, + 16 a uniform twiddle instead of the LDS tables), C3
# PFB_W5_TM=8/16/24 (the same bits).  C2 through gpu_ab.sh (HIP events), C3 through
# gpu_c3_kernel_ab.sh (rocprof).
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
if [ -n "${C2:-1}" ]; then
  V=""
  for v in 1 9 17 25; do for m in 0 3; do V="$V v${v}m$m:PFB_WAVE_V=$v,PFB_TIMING_MASK=$m"; done; done
  ROUNDS=${ROUNDS:-1} timeout -k 10 900 bash scripts/gpu_ab.sh $V > gpurun_out/ab.log 2>&1 || { rc=$?; tail -20 gpurun_out/ab.log; exit $rc; }
  cp gpurun_out/ab.jsonl gpurun_out/c2_masks.jsonl
  cat gpurun_out/ab.log
fi
if [ -n "${C3:-1}" ]; then
  V3=""
  for t in 0 8 16 24; do for m in 0 3; do V3="$V3 t${t}m$m:PFB_W5_TM=$t,PFB_TIMING_MASK=$m"; done; done
  ROUNDS=1 timeout -k 10 900 bash scripts/gpu_c3_kernel_ab.sh $V3 > gpurun_out/c3k.log 2>&1 || { rc=$?; tail -20 gpurun_out/c3k.log; exit $rc; }
  cat gpurun_out/c3k.log
fi
