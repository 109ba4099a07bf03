#!/bin/bash
# Round-5 validation: GPU tests, smoke, bench (C2 + synthesis_only + c3), TwoStage and LowCBF
# timings (bench_aux subset), the bench under rocprofv3.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/parity_errors.jsonl
PFB_PARITY_LOG=$GRAFT_REPO_ROOT/gpurun_out/parity_errors.jsonl timeout -k 10 900 \
    python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
timeout -k 10 600 python scripts/bench_aux.py --reps 10 --skip-mid > gpurun_out/bench_aux.jsonl 2> gpurun_out/bench_aux.err || exit $?
cut -c1-120 gpurun_out/bench_aux.jsonl
if [ -n "${PROF:-}" ]; then
  rm -rf gpurun_out/prof_bench
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o bench -- \
      python bench.py --steps 20 --warmup 3 > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err || exit $?
fi
if [ -n "${C3K:-}" ]; then
  ROUNDS=2 timeout -k 10 900 bash scripts/gpu_c3_kernel_ab.sh $C3K > gpurun_out/c3k.log 2>&1 || exit $?
  cat gpurun_out/c3k.log
fi
