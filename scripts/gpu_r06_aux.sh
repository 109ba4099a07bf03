#!/bin/bash
# Round 6: bench_aux on the final code (every secondary workload) and a kernel trace of the
# TwoStage cascade calls (GPU time per call vs the host-timed figure).
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python scripts/bench_aux.py --reps 10 > gpurun_out/bench_aux.jsonl 2> gpurun_out/bench_aux.err || { tail -5 gpurun_out/bench_aux.err; exit 3; }
cut -c1-140 gpurun_out/bench_aux.jsonl
cd /tmp
rm -rf $R/gpurun_out/prof_ts
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_ts -o ts -- \
    python3 $R/scripts/bench_aux.py --only-twostage --reps 20 > $R/gpurun_out/ts_prof.jsonl 2> $R/gpurun_out/ts_prof.err || exit 4
python3 - $R/gpurun_out/prof_ts/ts_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f'{float(r["AverageNs"])/1e3:8.1f} us x{r["Calls"]:>4} {r["Name"][:90]}')
PY
