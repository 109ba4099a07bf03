#!/bin/bash
# Second half of an end-of-round GPU session (the first is gpu_round.sh): secondary kernels
# (bench_aux), the C3 kernel trace, the PCIe-inclusive bench, FETCH/WRITE PMC passes of the
# C2 and C4 steps and of the C3 round trip (profiles/pmc_traffic.json records), SQ passes of
# the C2 and C3 steps, and the full C5 purity sweep.  Stops at the first failing step.
set -u
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python scripts/bench_aux.py --reps 10 > gpurun_out/bench_aux.jsonl 2> gpurun_out/bench_aux.err \
    || { echo "bench_aux failed"; tail -5 gpurun_out/bench_aux.err; exit 1; }
echo "bench_aux ok"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/c3prof -o run \
    -- python3 $R/scripts/bench_aux.py --only-mid --reps 5 > $R/gpurun_out/c3prof.log 2>&1 || exit $?
cd $R && echo "c3 profile ok"
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --e2e 1 --no-cpu-baseline > gpurun_out/bench_e2e.json 2> gpurun_out/bench_e2e.err \
    || exit $?
echo "e2e ok"
rm -rf gpurun_out/pmc_*
bash scripts/gpu_pmc.sh FETCH_SIZE WRITE_SIZE || exit $?
mv gpurun_out/pmc_1 gpurun_out/pmc_c2_fetch && mv gpurun_out/pmc_2 gpurun_out/pmc_c2_write
BENCH_ARGS="--workload c4" bash scripts/gpu_pmc.sh FETCH_SIZE WRITE_SIZE || exit $?
mv gpurun_out/pmc_1 gpurun_out/pmc_c4_fetch && mv gpurun_out/pmc_2 gpurun_out/pmc_c4_write
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic.json
python3 scripts/pmc_summary.py --json gpurun_out/pmc_traffic.json c2 gpurun_out/pmc_c2_fetch gpurun_out/pmc_c2_write > gpurun_out/pmc_c2_summary.txt
python3 scripts/pmc_summary.py --json gpurun_out/pmc_traffic.json c4 gpurun_out/pmc_c4_fetch gpurun_out/pmc_c4_write > gpurun_out/pmc_c4_summary.txt
PMC_PROG="scripts/bench_aux.py --only-mid --reps 2" bash scripts/gpu_pmc.sh FETCH_SIZE WRITE_SIZE || exit $?
mv gpurun_out/pmc_1 gpurun_out/pmc_c3_fetch && mv gpurun_out/pmc_2 gpurun_out/pmc_c3_write
python3 scripts/pmc_summary.py gpurun_out/pmc_c3_fetch gpurun_out/pmc_c3_write > gpurun_out/pmc_c3_summary.txt
bash scripts/gpu_pmc.sh "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
    "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" || exit $?
python3 scripts/pmc_summary.py gpurun_out/pmc_1 gpurun_out/pmc_2 > gpurun_out/pmc_c2_sq_summary.txt
rm -rf gpurun_out/pmc_1 gpurun_out/pmc_2
PMC_PROG="scripts/bench_aux.py --only-mid --reps 2" bash scripts/gpu_pmc.sh \
    "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
    "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" || exit $?
python3 scripts/pmc_summary.py gpurun_out/pmc_1 gpurun_out/pmc_2 > gpurun_out/pmc_c3_sq_summary.txt
echo "pmc ok"
timeout -k 10 400 python scripts/purity_sweep.py > gpurun_out/purity_sweep.jsonl 2> gpurun_out/purity_sweep.err || exit $?
tail -1 gpurun_out/purity_sweep.jsonl
