#!/bin/bash
# A/B of the N > 256 register-window FIR (C3): rows per loop iteration (PFB_FIR_ROWS),
# kernel times from rocprofv3.  Parity subset first, at every setting measured.
set -u
mkdir -p gpurun_out/abfir
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for u in ${ROWS:-3 2 1}; do
  PFB_FIR_ROWS=$u timeout -k 10 300 python -m pytest tests/test_gpu_parity.py tests/test_gpu_roundtrip.py -q -x \
      -p no:cacheprovider --timeout 120 -k "padded or generic or mid or 4096 or 512 or 1024 or separate_calls or c3_full" \
      > gpurun_out/abfir/pytest_$u.log 2>&1 || { tail -20 gpurun_out/abfir/pytest_$u.log; exit 1; }
  echo "rows=$u: $(tail -1 gpurun_out/abfir/pytest_$u.log)"
done
for u in ${ROWS:-3 2 1}; do
  cd /tmp && PFB_FIR_ROWS=$u timeout -k 10 240 rocprofv3 --kernel-trace --stats \
      --output-format csv -d $R/gpurun_out/abfir/p_$u -o run -- python3 $R/scripts/bench_aux.py --only-mid --reps 5 \
      > $R/gpurun_out/abfir/aux_$u.jsonl 2>/dev/null || exit $?
  cd $R
  echo "rows=$u"; grep -h roundtrip gpurun_out/abfir/aux_$u.jsonl | head -2
  python3 - "$R/gpurun_out/abfir/p_$u/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "pfb::" in r["Name"]:
        print("  ", r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
done
