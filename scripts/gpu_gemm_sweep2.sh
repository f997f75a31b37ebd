# GPU: tools/gemm_bench tile x split sweeps over the D0 shapes: BN + swish view (mode 1) and the
# gradient view (mode 3)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ONLY=0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15,16,17,18,19,20,21,22,23
GEMM_ONLY=$ONLY GEMM_SWEEP=1 GEMM_MODE=1 timeout -k 10 400 tools/gemm_bench > gpurun_out/sw_m1.txt 2>&1; rc=$?; echo "m1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
GEMM_ONLY=$ONLY GEMM_SWEEP=1 GEMM_MODE=3 timeout -k 10 400 tools/gemm_bench > gpurun_out/sw_m3.txt 2>&1; echo "m3 rc=$?"
