#!/bin/bash
# Round 6: C3 work session — C3 / padded / 4096 GPU tests, the copy-shape probe, per-kernel
# C3 A/B of experiments-build variants (gpu_c3_kernel_ab.sh; VARIANTS), FETCH/WRITE PMC passes
# of the C3 round trip (release build).
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf \
    -k "${K:-c3 or mid or padded or 4096 or rowfft or sharding}" > gpurun_out/pytest_c3.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_c3.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ -n "${PROBE:-1}" ] && [ -x scripts/copy_probe ]; then
  timeout -k 10 300 scripts/copy_probe > gpurun_out/copy_probe.jsonl 2>&1 || exit $?
  cat gpurun_out/copy_probe.jsonl
fi
if [ -n "${VARIANTS:-}" ]; then
  ROUNDS=${ROUNDS:-2} timeout -k 10 900 bash scripts/gpu_c3_kernel_ab.sh $VARIANTS > gpurun_out/c3k.log 2>&1 || exit $?
  cat gpurun_out/c3k.log
fi
if [ -n "${PMC:-1}" ]; then
  WORKLOADS=c3 timeout -k 10 600 bash scripts/gpu_pmc_r05.sh > gpurun_out/pmc.log 2>&1 || exit $?
  cat gpurun_out/pmc.log
  python3 scripts/pmc_summary.py gpurun_out/pmc_c3_* > gpurun_out/pmc_c3_summary.txt 2>&1
  cat gpurun_out/pmc_c3_summary.txt
fi
