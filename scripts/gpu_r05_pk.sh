# GPU: the packed-FP32 fix.  Concurrent-step checksums (D4 bf16 1024^2 x 4, D0 bf16 1024^2 x 4) with
# the default (no packed FP32) build; one-stream gradients of both builds; C2 and C4 timing A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
ck() { timeout -k 10 300 python -u scripts/diag_cksum.py "$@"; }
ck efficientdet-d4 1024 bf16 16 > gpurun_out/pk_d4.log 2>&1 && echo "d4 new: $(grep -h 'differing concurrent' gpurun_out/pk_d4.log)" && \
PHX_LIB=libphx_pk.so ck efficientdet-d4 1024 bf16 4 > gpurun_out/pk_d4_old.log 2>&1 && echo "d4 pk: $(grep -h 'differing concurrent' gpurun_out/pk_d4_old.log)" && \
python -c "
import numpy as np
a=np.load('gpurun_out/g0_libphx_pk.so.npy'); b=np.load('gpurun_out/g0_libphx.so.npy')
print('one-stream D4 bf16 gradients, packed vs unpacked build: bit-identical', np.array_equal(a.view(np.uint32), b.view(np.uint32)), 'max|d|', float(np.abs(a-b).max()))
" && \
ck efficientdet-d0 1024 bf16 12 > gpurun_out/pk_d0.log 2>&1 && echo "d0 bf16 new: $(grep -h 'differing concurrent' gpurun_out/pk_d0.log)" || exit 1
for r in 1 2; do
  for lib in libphx.so libphx_pk.so; do
    PHX_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary > gpurun_out/pk_c2_$lib.json 2>/dev/null || exit 1
    echo "C2 $lib: $(python -c "import json;d=json.load(open('gpurun_out/pk_c2_$lib.json'));print(d['ms_per_step'], d['value'])")"
    PHX_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --model efficientdet-d4 --image-size 1024 --batch 4 --dtype bf16 --steps 60 > gpurun_out/pk_c4_$lib.json 2>/dev/null || exit 1
    echo "C4 $lib: $(python -c "import json;d=json.load(open('gpurun_out/pk_c4_$lib.json'));print(d['ms_per_step'], d['value'])")"
  done
done
