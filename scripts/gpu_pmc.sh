# GPU: HBM traffic of the hot kernels from PMC counters, one counter per pass (FETCH_SIZE and
# WRITE_SIZE do not fit one TCC pass; MI355X_MICROARCH.md "rocprofv3 PMC slots"), kernel-trace only.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
RX=${PMC_RX:-'k_gemm|k_dw_|k_sep_|k_colred|k_bn_finalize|k_se_mlp|k_ew_gstats'}
CMD=${PMC_CMD:-"python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-secondary"}
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" -d gpurun_out/pmc_fetch -o run \
  --output-format csv -- $CMD > gpurun_out/pmc_fetch.log 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" -d gpurun_out/pmc_write -o run \
  --output-format csv -- $CMD > gpurun_out/pmc_write.log 2>&1
echo "write rc=$?"
