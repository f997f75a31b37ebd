# GPU: tools/gemm_bench with and without the statistics epilogue (the D0 shapes)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 tools/gemm_bench > gpurun_out/gb_stats.txt 2>&1; rc=$?; echo "stats rc=$rc"; [ $rc -eq 0 ] || exit $rc
GEMM_NOSTATS=1 timeout -k 10 200 tools/gemm_bench > gpurun_out/gb_nostats.txt 2>&1; echo "nostats rc=$?"
