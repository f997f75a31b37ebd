# GPU: D4 256^2 bf16 step deviations under three GEMM plans (scripts/diag_bf16_wsk.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/diag_bf16_oracle.npz
PHX_GEMM_WSK_BF16=0 timeout -k 10 400 python -u scripts/diag_bf16_wsk.py || exit $?
PHX_GEMM_WSK_BF16=1 timeout -k 10 200 python -u scripts/diag_bf16_wsk.py || exit $?
PHX_GEMM_WSK=0 timeout -k 10 200 python -u scripts/diag_bf16_wsk.py || exit $?
