#!/bin/bash
# PMC counter passes over a short bench run (one counter group per process, --pmc only).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $ROOT/gpurun_out
export TMPDIR=/tmp
cd /tmp
STEPS=${STEPS:-3}
timeout -k 10 120 rocprofv3 -L > $ROOT/gpurun_out/rocprof_counters.txt 2>&1 || true
i=0
SETS=("$@")
if [ ${#SETS[@]} -eq 0 ]; then SETS=("FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"); fi
for set in "${SETS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $ROOT/gpurun_out/pmc_$i -o pmc \
      -- python3 $ROOT/${PMC_PROG:-bench.py --steps $STEPS --warmup 1 --no-cpu-baseline --inflight 1} ${BENCH_ARGS:-} > $ROOT/gpurun_out/pmc_$i.log 2>&1
  rc=$?
  echo "pmc pass $i ($set) rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 $ROOT/gpurun_out/pmc_$i.log; exit $rc; fi
done
