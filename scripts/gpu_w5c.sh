#!/bin/bash
# SKA-Mid wave synthesis with the lower-conflict LDS layout: parity subset, then C3 round trip
# interleaved with the previous layout's library (lib/libpfb_hip_prev.so), and the kernel
# trace + LDS counters of the new one.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread -rf -k "nf512 or c3 or 4096 or baseline_shapes or mid or split" > gpurun_out/pytest_w5c.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_w5c.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; exit $rc; fi
: > gpurun_out/c3_layout.jsonl
for round in 1 2 3; do
  for v in new prev; do
    lib=$R/ska-pst-dsp-model_amd/lib/libpfb_hip.so; [ $v = prev ] && lib=$R/ska-pst-dsp-model_amd/lib/libpfb_hip_prev.so
    PFB_HIP_LIB=$lib timeout -k 10 200 python scripts/bench_aux.py --only-mid --reps 5 > gpurun_out/c3l.json 2> gpurun_out/c3l.err || { tail -3 gpurun_out/c3l.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/c3l.json')); print(json.dumps({'tag': '$v', 'ms': d['ms']}))" | tee -a gpurun_out/c3_layout.jsonl
  done
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/c3prof -o run \
    -- python3 $R/scripts/bench_aux.py --only-mid --reps 5 > $R/gpurun_out/c3prof.log 2>&1 || exit $?
cd $R && python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/c3prof/run_kernel_stats.csv')):
    if 'pfb' in r['Name']: print(r['Name'][:90], r['Calls'], round(float(r['AverageNs'])/1e3,1),'us')
"
PMC_PROG="scripts/bench_aux.py --only-mid --reps 2" bash scripts/gpu_pmc.sh "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" > /dev/null || exit $?
python3 scripts/pmc_summary.py gpurun_out/pmc_1 | grep -A1 synth_wave512
