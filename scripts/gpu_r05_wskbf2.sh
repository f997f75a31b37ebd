# GPU: bf16 wave-split-K tile sweep on the D4 deep-K shapes (SE view, gradient view)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in 2 3; do
  GEMM_ONLY=24,25,8,17 GEMM_WSK=1 GEMM_BF16=1 GEMM_MODE=$m timeout -k 10 120 tools/gemm_bench > gpurun_out/wskbf_m$m.txt 2>&1
  rc=$?; echo "wsk bf16 mode $m rc=$rc"; grep -E "^wsk" gpurun_out/wskbf_m$m.txt; [ $rc -eq 0 ] || exit $rc
done
