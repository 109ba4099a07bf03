#!/bin/bash
# Round-6 GPU session script: every step under its own time limit, stop at the first
# failure that is not a test failure.  STEPS picks the steps (default: tests smoke bench):
#   tests   — pytest -m gpu (PFB_PARITY_LOG -> gpurun_out/parity_errors.jsonl); K=<expr> filters
#   smoke   — __graft_entry__.smoke()
#   bench   — bench.py --steps 20 --warmup 3
#   aux     — scripts/bench_aux.py (TwoStage, LowCBF, DADA, ...)
#   prof    — the bench under rocprofv3 --kernel-trace --stats
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-"tests smoke bench"}
for step in $STEPS; do
  case $step in
    tests)
      rm -f gpurun_out/parity_errors.jsonl
      KARG=()
      if [ -n "${K:-}" ]; then KARG=(-k "$K"); fi
      PFB_PARITY_LOG=$GRAFT_REPO_ROOT/gpurun_out/parity_errors.jsonl timeout -k 10 1000 \
        python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf \
        "${KARG[@]}" > gpurun_out/pytest_gpu.log 2>&1
      rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
      if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
      ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
      cat gpurun_out/smoke.log
      ;;
    bench)
      timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
      cut -c1-400 gpurun_out/bench.json
      ;;
    aux)
      timeout -k 10 600 python scripts/bench_aux.py --reps 10 ${AUXARGS:-} > gpurun_out/bench_aux.jsonl 2> gpurun_out/bench_aux.err || exit $?
      cut -c1-160 gpurun_out/bench_aux.jsonl
      ;;
    prof)
      rm -rf gpurun_out/prof_bench
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o bench -- \
        python bench.py --steps 20 --warmup 3 > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err || exit $?
      ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
