#!/bin/bash
# Development iteration on one GPU box: GPU parity tests (stop at the first failure), the
# C2 bench, and a kernel trace of a short bench run.  Each GPU step has its own limit and
# nothing else starts after a fault, abort or timeout.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rm -f gpurun_out/parity_errors.jsonl
PFB_PARITY_LOG=$R/gpurun_out/parity_errors.jsonl timeout -k 10 600 \
    python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -rf \
    ${PT_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -8 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; if [ $rc -ne 0 ]; then echo "bench rc=$rc"; tail -5 gpurun_out/bench.err; exit $rc; fi
python3 -c "import json; d=json.load(open('gpurun_out/bench.json')); print('C2', d['value'], d['ms_per_step'], {k: (v['kernel'][:60], round(v['avg_ms']*1e3,1)) for k,v in d['kernels'].items()})"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run \
    -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof.log 2>&1
rc=$?; cd $R
if [ $rc -ne 0 ]; then echo "rocprof rc=$rc"; tail -5 gpurun_out/prof.log; exit $rc; fi
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/prof/run_kernel_stats.csv')):
    if 'pfb' in r['Name']: print(r['Name'][:90], r['Calls'], round(float(r['AverageNs'])/1e3,1),'us')
"
