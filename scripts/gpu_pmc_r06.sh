#!/bin/bash
# Round 6: FETCH_SIZE / WRITE_SIZE rocprofv3 passes (one counter per process, --pmc only)
# over scripts/pmc_prog.py for every workload bench.py reports a `traffic` for, merged into
# gpurun_out/pmc_traffic.json under bench.py's workload keys (c2, c4, synthesis_only_p1,
# synthesis_only_p2, c3); SQ passes (SQ=1) for the C2 / C3 kernels' instruction mix.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $ROOT/gpurun_out
export TMPDIR=/tmp
cd /tmp
declare -A KEY=([c2]=c2 [c4]=c4 [c2syn]=synthesis_only_p1 [c4syn]=synthesis_only_p2 [c3]=c3 [c3p2]=c3_p2)
SETS=("FETCH_SIZE" "WRITE_SIZE")
if [ -n "${SQ:-}" ]; then
  SETS+=("SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE")
fi
rm -f $ROOT/gpurun_out/pmc_traffic.json
for wl in ${WORKLOADS:-c2 c4 c2syn c4syn c3}; do
  i=0
  for set in "${SETS[@]}"; do
    i=$((i+1))
    rm -rf $ROOT/gpurun_out/pmc_${wl}_$i
    timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $ROOT/gpurun_out/pmc_${wl}_$i -o pmc \
        -- python3 $ROOT/scripts/pmc_prog.py --workload $wl > $ROOT/gpurun_out/pmc_${wl}_$i.log 2>&1
    rc=$?
    echo "pmc $wl pass $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -20 $ROOT/gpurun_out/pmc_${wl}_$i.log; exit $rc; fi
  done
  python3 $ROOT/scripts/pmc_summary.py --json $ROOT/gpurun_out/pmc_traffic.json ${KEY[$wl]} $ROOT/gpurun_out/pmc_${wl}_* \
      > $ROOT/gpurun_out/pmc_${wl}_summary.txt 2>&1
  cat $ROOT/gpurun_out/pmc_${wl}_summary.txt
done
