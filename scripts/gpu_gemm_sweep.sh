# GPU: tile-configuration x split-K sweeps of tools/gemm_bench over the D0 1x1-conv shapes:
# raw A (mode 0), BN + swish view (mode 1), gradient view (mode 3), and mode 1 on bf16 cores
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in 0 1 3; do
  GEMM_ONLY=0,3,4,5,6,7,8,9,10,11,12,13,14,16 GEMM_SWEEP=1 GEMM_MODE=$m timeout -k 10 300 tools/gemm_bench > gpurun_out/gemm_sweep_m$m.txt 2>&1
  rc=$?; echo "sweep mode $m rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
GEMM_ONLY=0,3,4,5,6,7,8,9,10,11,12,13,14,16 GEMM_SWEEP=1 GEMM_MODE=1 GEMM_BF16=1 timeout -k 10 300 tools/gemm_bench > gpurun_out/gemm_sweep_m1bf.txt 2>&1
echo "sweep bf16 rc=$?"
