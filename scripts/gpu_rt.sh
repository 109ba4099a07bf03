#!/bin/bash
# GPU tests (round trip + parity), then a short bench sweep.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_roundtrip.py tests/test_gpu_parity.py -m gpu -x -q \
    -p no:cacheprovider --timeout 300 --timeout-method thread -rf > gpurun_out/pytest_rt.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_rt.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash scripts/gpu_sweep.sh "serial python bench.py --steps 20 --pipeline 0" \
  "oldana env PFB_ANALYSIS_NO_STREAM=1 python bench.py --steps 20 --pipeline 0" \
  "rt64 python bench.py --steps 20" \
  "rt256 env PFB_RT_CHUNK_BLOCKS=256 python bench.py --steps 20"
