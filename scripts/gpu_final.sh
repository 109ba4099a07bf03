#!/bin/bash
# End-of-round GPU session: parity tests (error statistics), smoke, C2 bench + C4 unit bench
# + kernel trace (gpu_round.sh), then the secondary kernels, the C3 kernel trace, the
# PCIe-inclusive bench and the FETCH/WRITE PMC passes of the C2 step and of the C3 round trip.
set -u
R=$GRAFT_REPO_ROOT
bash scripts/gpu_round.sh || exit $?
cd $R
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
# roofline.traffic records (copied to profiles/pmc_traffic.json after the run)
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic.json
python3 scripts/pmc_summary.py --json gpurun_out/pmc_traffic.json c2 gpurun_out/pmc_c2_fetch gpurun_out/pmc_c2_write > /dev/null
python3 scripts/pmc_summary.py --json gpurun_out/pmc_traffic.json c4 gpurun_out/pmc_c4_fetch gpurun_out/pmc_c4_write > /dev/null
PMC_PROG="scripts/bench_aux.py --only-mid --reps 2" bash scripts/gpu_pmc.sh FETCH_SIZE WRITE_SIZE || exit $?
mv gpurun_out/pmc_1 gpurun_out/pmc_c3_fetch && mv gpurun_out/pmc_2 gpurun_out/pmc_c3_write
echo "pmc ok"
