# GPU: is the concurrent-step difference cache-line sharing between small buffers?  Allocation
# addresses, then the checksum diagnosis with 256-B guard bands around every executor buffer.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
export PHX_BF16_HALF_FORK=0
PHX_ALLOC_LOG=1 timeout -k 10 300 python -u scripts/diag_cksum.py efficientdet-d4 1024 bf16 2 > gpurun_out/cksum_alloc.log 2>&1
echo "alloc-log rc=$?"
grep "phx alloc" gpurun_out/cksum_alloc.log | python -c "
import sys
a=[(int(l.split()[2],16),int(l.split()[3])) for l in sys.stdin]
a.sort()
small=[x for x in a if x[1]<4096]
print('allocations',len(a),'small(<4KB)',len(small))
gaps=[(b[0]-(p[0]+p[1]), p, b) for p,b in zip(a,a[1:])]
shared=[g for g in gaps if (g[1][0]+g[1][1]-1)//128 == g[2][0]//128]
print('adjacent pairs sharing a 128-B line:', len(shared))
for g in shared[:10]: print('  %x+%d | %x+%d' % (g[1][0], g[1][1], g[2][0], g[2][1]))
print('alignments of small allocations:', sorted(set(x[0] % 4096 for x in small))[:20])
"
PHX_GUARD_BYTES=256 timeout -k 10 300 python -u scripts/diag_cksum.py efficientdet-d4 1024 bf16 12 > gpurun_out/cksum_guard.log 2>&1
echo "guard rc=$?"; grep -v amdgpu.ids gpurun_out/cksum_guard.log | grep -v "phx guard" | tail -30
