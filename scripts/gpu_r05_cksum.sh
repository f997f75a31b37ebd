# GPU: op-by-op checksums of concurrent vs one-stream steps (scripts/diag_cksum.py), D4 bf16 1024^2 x 4 with
# the side pass forking at stage 6 (the round-4 half-ops clamp off), then C2's D0 512^2 x 16 fp32.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
export PHX_BF16_HALF_FORK=0
timeout -k 10 300 python -u scripts/diag_cksum.py efficientdet-d4 1024 bf16 12 > gpurun_out/cksum_d4.log 2>&1
echo "d4 rc=$?"; grep -v amdgpu.ids gpurun_out/cksum_d4.log | tail -60
