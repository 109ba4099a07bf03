#!/bin/bash
# C3 synthesis timing-mask breakdown (results invalid by design: HBM accesses dropped).
set -u
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
for m in ${MASKS:-0 1 2 4 7}; do
  cd /tmp && PFB_TIMING_MASK=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/m$m -o run \
      -- python3 $R/scripts/bench_aux.py --only-mid --reps 3 > $R/gpurun_out/m$m.log 2>&1 || exit $?
  cd $R && python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/m$m/run_kernel_stats.csv')):
    if 'synth' in r['Name'] or 'fir_' in r['Name'] or 'row_fft' in r['Name']: print('mask $m', r['Name'][:40], round(float(r['AverageNs'])/1e3,1),'us')
"
done
