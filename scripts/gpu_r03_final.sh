# GPU: round-3 final evidence — rocprofv3 kernel-trace summary of the bench command, HBM traffic
# (FETCH_SIZE, WRITE_SIZE: one PMC pass each), then the C2 (default bench: CPU baseline and the
# first-pass line), C4 and C5 lines.  Stops at the first failing step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o run --output-format csv -- \
  python bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-secondary > gpurun_out/prof_final.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
RX2='k_gemm|k_dw_|k_colred|k_bn_finalize|k_se_mlp|k_ew_gstats'
CMD2="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-secondary"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX2" -d gpurun_out/pmc_fetch -o run \
  --output-format csv -- $CMD2 > gpurun_out/pmc_fetch.log 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX2" -d gpurun_out/pmc_write -o run \
  --output-format csv -- $CMD2 > gpurun_out/pmc_write.log 2>&1
rc=$?; echo "write rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r03_lines2.sh
