# GPU: tools/gemm_bench over the D0 1x1-conv shapes and three large ones, then one PMC pass
# (MFMA busy / wait / issue counters) over the 65536x512x512 shape
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 tools/gemm_bench > gpurun_out/gemm_bench.txt 2>&1
rc=$?; echo "gemm_bench rc=$rc"; cat gpurun_out/gemm_bench.txt | tail -20
[ $rc -eq 0 ] || exit $rc
GEMM_ONLY=14,9,10 timeout -s KILL 60 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
  --kernel-include-regex "k_gemm2" -d gpurun_out/pmc_gemm -o run --output-format csv -- tools/gemm_bench > gpurun_out/pmc_gemm.log 2>&1
echo "pmc rc=$?"
