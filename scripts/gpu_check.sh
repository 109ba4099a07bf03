#!/bin/bash
# Full GPU test suite, then C2 bench and the C3 round trip (bench_aux --only-mid), then the
# LDS bank-conflict counters of a short C2 bench and of the C3 round trip.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 800 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf \
    > gpurun_out/pt.log 2>&1
rc=$?; tail -6 gpurun_out/pt.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench.json')); print('C2', d['value'], d['ms_per_step'], {k: round(v['avg_ms']*1e3,1) for k,v in d['kernels'].items()})"
timeout -k 10 200 python scripts/bench_aux.py --only-mid --reps 10 > gpurun_out/c3.jsonl 2> gpurun_out/c3.err || exit $?
cat gpurun_out/c3.jsonl
if [ -n "${PMC:-}" ]; then
  bash scripts/gpu_pmc.sh "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" > gpurun_out/pmc.log 2>&1 || exit $?
  mv gpurun_out/pmc_1 gpurun_out/pmc_c2
  PMC_PROG="scripts/bench_aux.py --only-mid --reps 2" bash scripts/gpu_pmc.sh "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" >> gpurun_out/pmc.log 2>&1 || exit $?
  mv gpurun_out/pmc_1 gpurun_out/pmc_c3
  python3 scripts/pmc_summary.py gpurun_out/pmc_c2 | grep -E "==|bank"
  python3 scripts/pmc_summary.py gpurun_out/pmc_c3 | grep -E "==|bank"
fi
