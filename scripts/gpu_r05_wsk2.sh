# GPU: forced wave-split-K tiles on the unsplit mid-K D0 shapes (BN view), against the default plan
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in 1 3; do
  GEMM_ONLY=9,7,15,14,5 GEMM_WSK=1 GEMM_MODE=$m timeout -k 10 120 tools/gemm_bench > gpurun_out/wsk2_m$m.txt 2>&1
  rc=$?; echo "wsk2 mode $m rc=$rc"; grep -E "^wsk" gpurun_out/wsk2_m$m.txt; [ $rc -eq 0 ] || exit $rc
done
