#!/bin/bash
# Round-5 probes: HBM streaming ceilings (copy / read / write) and a kernel-trace profile
# of the TwoStage cascade stream call.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
: timeout -k 10 300 python scripts/hbm_probe.py > gpurun_out/hbm_probe.jsonl 2> gpurun_out/hbm_probe.err || exit $?
: cat
rm -rf gpurun_out/prof_ts
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ts -o ts -- \
    python scripts/bench_aux.py --only-twostage --reps 20 > gpurun_out/ts.log 2>&1 || exit $?
cat gpurun_out/ts.log | tail -3
f=$(find gpurun_out/prof_ts -name "*kernel_stats.csv" | head -1); cut -d, -f1-5 "$f" | head -15
t=$(find gpurun_out/prof_ts -name "*kernel_trace.csv" | head -1)
python3 - "$t" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
last = rows[-12:]
t0 = int(last[0]["Start_Timestamp"])
for r in last:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f'{s/1e3:9.1f} {e/1e3:9.1f} {(e-s)/1e3:7.1f}  {r["Kernel_Name"][:90]}')
PY
