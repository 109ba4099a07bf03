#!/bin/bash
# A/B of library env knobs on C3 (bench_aux --only-mid under rocprofv3 --kernel-trace),
# each setting after the C3-relevant parity subset.  Args: "name VAR=value ..." items
# ("name" alone = defaults).
set -u
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for item in "$@"; do
  set -- $item
  nm=$1; shift
  ( if [ $# -gt 0 ]; then export "$@"; fi
    timeout -k 10 300 python -m pytest tests/test_gpu_parity.py tests/test_gpu_roundtrip.py -q -x \
      -p no:cacheprovider --timeout 120 -k "padded or generic or mid or 4096 or 512 or 1024 or separate_calls or c3_full or synthesis" \
      > gpurun_out/ab/pytest_$nm.log 2>&1 ) || { tail -20 gpurun_out/ab/pytest_$nm.log; exit 1; }
  echo "$nm: $(tail -1 gpurun_out/ab/pytest_$nm.log)"
  ( if [ $# -gt 0 ]; then export "$@"; fi; cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats \
      --output-format csv -d $R/gpurun_out/ab/p_$nm -o run -- python3 $R/scripts/bench_aux.py --only-mid --reps 5 \
      > $R/gpurun_out/ab/aux_$nm.jsonl 2>/dev/null ) || exit $?
  grep -h roundtrip gpurun_out/ab/aux_$nm.jsonl | head -2
  python3 - "$R/gpurun_out/ab/p_$nm/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "pfb::" in r["Name"]:
        print("  ", r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
done
