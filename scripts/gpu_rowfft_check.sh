set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread -k "c3 or mid or nf512 or sharding or padded" > gpurun_out/pytest_rf.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_rf.log; [ $rc -ne 0 ] && exit $rc
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_rf -o pmc -- python3 $GRAFT_REPO_ROOT/scripts/pmc_prog.py --workload c3 > $GRAFT_REPO_ROOT/gpurun_out/pmc_rf.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
python3 scripts/pmc_summary.py gpurun_out/pmc_rf | grep -A8 row_fft4096
timeout -k 10 300 python scripts/bench_aux.py --only-mid --reps 10 | cut -c1-100
