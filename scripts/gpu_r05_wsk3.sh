# GPU: forced wave-split-K tiles on the small BiFPN-level GEMMs (K 64, few tiles) against the default plan
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in 0 1; do
  GEMM_ONLY=12,28,29,11,6 GEMM_WSK=1 GEMM_MODE=$m timeout -k 10 120 tools/gemm_bench > gpurun_out/wsk3_m$m.txt 2>&1
  rc=$?; echo "wsk3 mode $m rc=$rc"; grep -E "^wsk" gpurun_out/wsk3_m$m.txt; [ $rc -eq 0 ] || exit $rc
done
