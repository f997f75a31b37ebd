# GPU: which configurations show the concurrent-step difference?  D4 bf16 without drop connect,
# D4 fp32 (512^2: its fp32 workspace at 1024^2 x 4 is large), D1 fp32, D0 bf16 1024^2.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
export PHX_BF16_HALF_FORK=0
run() { name=$1; shift; timeout -k 10 300 "$@" > gpurun_out/which_$name.log 2>&1; rc=$?; echo "$name rc=$rc: $(grep -h 'differing concurrent' gpurun_out/which_$name.log)"; return $rc; }
PHX_LIB=libphx_nopk.so run d4bf16_nopk python -u scripts/diag_cksum.py efficientdet-d4 1024 bf16 16 && \
PHX_NO_DROP=1 run d4bf16_nodrop python -u scripts/diag_cksum.py efficientdet-d4 1024 bf16 12 && \
run d4f32_512 python -u scripts/diag_cksum.py efficientdet-d4 512 f32 12 && \
run d4bf16_512 python -u scripts/diag_cksum.py efficientdet-d4 512 bf16 12 && \
run d1f32 python -u scripts/diag_cksum.py efficientdet-d1 640 f32 12 && \
run d0bf16 python -u scripts/diag_cksum.py efficientdet-d0 1024 bf16 12
for f in gpurun_out/which_*.log; do echo "== $f"; grep -A2 "^step" $f | grep "\[" | head -4; done
