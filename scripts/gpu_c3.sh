#!/bin/bash
# C3 (SKA-Mid) A/B: round-trip tests, then bench_aux --only-mid with the default and an
# alternative environment (AB_ENV), then a kernel trace of the C3 round trip.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    -k "${PT_K:-roundtrip}" > gpurun_out/pt.log 2>&1
rc=$?; tail -4 gpurun_out/pt.log
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2; do
  timeout -k 10 200 python scripts/bench_aux.py --only-mid --reps 10 > gpurun_out/c3_new_$i.jsonl 2> gpurun_out/c3.err || exit $?
  cat gpurun_out/c3_new_$i.jsonl
  env ${AB_ENV:-PFB_NONE=1} timeout -k 10 200 python scripts/bench_aux.py --only-mid --reps 10 > gpurun_out/c3_old_$i.jsonl 2> gpurun_out/c3.err || exit $?
  echo "alt (${AB_ENV:-}):"; cat gpurun_out/c3_old_$i.jsonl
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/c3prof -o run \
    -- python3 $R/scripts/bench_aux.py --only-mid --reps 5 > $R/gpurun_out/c3prof.log 2>&1 || exit $?
cd $R && python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/c3prof/run_kernel_stats.csv')):
    if 'pfb' in r['Name']: print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,1),'us')
"
