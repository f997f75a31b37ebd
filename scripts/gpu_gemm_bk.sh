# GPU: gemm_bench with fp32 K-chunks of 16 (libphx.so) and 32 (libphx_bk.so), planned configs (mode 0)
# and a mode-1 (BN + swish view) tile sweep over the MFMA-heavy shapes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 tools/gemm_bench > gpurun_out/gb16.txt 2>&1; rc=$?; echo "bk16 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 tools/gemm_bench_bk > gpurun_out/gb32.txt 2>&1; rc=$?; echo "bk32 rc=$rc"; [ $rc -eq 0 ] || exit $rc
GEMM_ONLY=5,7,9,10,13 GEMM_SWEEP=1 GEMM_MODE=1 timeout -k 10 300 tools/gemm_bench > gpurun_out/gb16_sw.txt 2>&1; echo "sw16 rc=$?"
GEMM_ONLY=5,7,9,10,13 GEMM_SWEEP=1 GEMM_MODE=1 timeout -k 10 300 tools/gemm_bench_bk > gpurun_out/gb32_sw.txt 2>&1; echo "sw32 rc=$?"
