#!/bin/bash
# Round 6: padded FilterBank rows written straight into the caller's buffer (no staging
# copy) — the filterbank / cascade / padded GPU tests and the cascade's kernel trace.
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -rf \
    -k "filterbank or two_stage or padded or mid or stream or sgcht or sharding" > gpurun_out/pytest_padfb.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_padfb.log
if [ $rc -ne 0 ]; then exit 3; fi
cd /tmp
rm -rf $R/gpurun_out/prof_ts2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_ts2 -o ts -- \
    python3 $R/scripts/bench_aux.py --only-twostage --reps 20 > $R/gpurun_out/ts2.jsonl 2> $R/gpurun_out/ts2.err || exit 4
cut -c1-160 $R/gpurun_out/ts2.jsonl
python3 - $R/gpurun_out/prof_ts2/ts_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f'{float(r["AverageNs"])/1e3:8.1f} us x{r["Calls"]:>4} {r["Name"][:90]}')
PY
