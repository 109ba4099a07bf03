#!/bin/bash
# Round-5 GPU session: the GPU test suite (parity errors logged), smoke, bench (C2 headline +
# synthesis_only + c3 keys), then C3 A/B variants of the experiments build (AB="tag:ENV=..").
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/parity_errors.jsonl
PFB_PARITY_LOG=$GRAFT_REPO_ROOT/gpurun_out/parity_errors.jsonl timeout -k 10 900 \
    python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/bench.err; exit $rc; fi
if [ -n "${AB:-}" ]; then
  ROUNDS=${ROUNDS:-2} timeout -k 10 900 bash scripts/gpu_c3_ab.sh $AB > gpurun_out/c3_ab.log 2>&1
  rc=$?; echo "c3 ab rc=$rc"; tail -3 gpurun_out/c3_ab.log; [ $rc -ne 0 ] && exit $rc
fi
if [ -n "${PROF:-}" ]; then
  rm -rf gpurun_out/prof_bench
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o bench -- \
      python bench.py --steps 20 --warmup 3 > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err
  rc=$?; echo "bench under rocprof rc=$rc"; exit $rc
fi
