#!/bin/bash
# PMC counter passes (one counter group per rocprofv3 process, --pmc only) over
# scripts/pmc_prog.py for each workload; CSVs in gpurun_out/pmc_<workload>_<pass>.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $ROOT/gpurun_out
export TMPDIR=/tmp
cd /tmp
SETS=("FETCH_SIZE" "WRITE_SIZE" \
      "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
      "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE")
for wl in ${WORKLOADS:-c2 c2syn c3}; do
  i=0
  for set in "${SETS[@]}"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $ROOT/gpurun_out/pmc_${wl}_$i -o pmc \
        -- python3 $ROOT/scripts/pmc_prog.py --workload $wl > $ROOT/gpurun_out/pmc_${wl}_$i.log 2>&1
    rc=$?
    echo "pmc $wl pass $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -20 $ROOT/gpurun_out/pmc_${wl}_$i.log; exit $rc; fi
  done
done
