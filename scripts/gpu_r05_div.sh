# GPU: the drop-connect division fix.  (1) div_surv == n / d bit for bit; (2) concurrent vs one-stream
# checksums with the plain division (libphx_hwdiv.so) and with div_surv (libphx.so); (3) the one-stream
# gradients of both builds equal.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
export PHX_BF16_HALF_FORK=0
mkdir -p gpurun_out
timeout -k 10 120 ./tools/div_check && \
PHX_LIB=libphx_hwdiv.so timeout -k 10 300 python -u scripts/diag_cksum.py efficientdet-d4 1024 bf16 12 > gpurun_out/div_hw.log 2>&1 && \
timeout -k 10 300 python -u scripts/diag_cksum.py efficientdet-d4 1024 bf16 16 > gpurun_out/div_new.log 2>&1
echo "rc=$?"
grep -h "differing concurrent\|one-stream rerun" gpurun_out/div_hw.log gpurun_out/div_new.log
python -c "
import numpy as np
a=np.load('gpurun_out/g0_libphx_hwdiv.so.npy'); b=np.load('gpurun_out/g0_libphx.so.npy')
print('one-stream gradients of the two builds bit-identical:', np.array_equal(a.view(np.uint32), b.view(np.uint32)))
"
