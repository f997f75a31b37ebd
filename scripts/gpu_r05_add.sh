# GPU: where does a concurrent step's residual-add output differ (scripts/diag_add.py)?
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
export PHX_BF16_HALF_FORK=0
timeout -k 10 300 python -u scripts/diag_add.py 10 > gpurun_out/diag_add.log 2>&1
echo "rc=$?"; grep -v amdgpu.ids gpurun_out/diag_add.log | tail -60
