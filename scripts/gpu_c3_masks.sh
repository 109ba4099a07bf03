set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export TMPDIR=/tmp
cd /tmp
for m in 0 1 2 3; do
  PFB_HIP_LIB=$R/ska-pst-dsp-model_amd/lib/libpfb_hip_exp.so PFB_TIMING_MASK=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/c3mask$m -o run -- python3 $R/scripts/bench_aux.py --only-mid --reps 5 > $R/gpurun_out/c3mask$m.log 2>&1 || exit $?
  echo "mask $m"; grep -E "fir_lds|row_fft|wave512" $R/gpurun_out/c3mask$m/run_kernel_stats.csv | cut -d, -f1-4
done
