# GPU (round 6): the 16x16 register GEMM (two chunks in flight) for fp32 outputs up to 32 wide
# (PHX_GEMM1_MAXN=32) against the 32x32 LDS-tiled kernel (default 16): the N <= 32 launch groups
# (tools/shape_prof.py), an alternating C2 bench A/B, then the full -m gpu suite with the knob set
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for V in 16 32; do
  PHX_GEMM1_MAXN=$V timeout -k 10 200 python tools/shape_prof.py --top 300 > gpurun_out/maxn_shapes_$V.txt 2>&1 || { tail -5 gpurun_out/maxn_shapes_$V.txt; exit 3; }
  echo "MAXN=$V"; grep -E "gemm .* N=(16|24|32) " gpurun_out/maxn_shapes_$V.txt || true
done
for r in 1 2 3; do
  for V in 16 32; do
    PHX_GEMM1_MAXN=$V timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --no-profile > gpurun_out/maxn_ab_$V.json 2>gpurun_out/maxn_ab_$V.err || exit 3
    echo "round $r MAXN=$V: $(python -c "import json;d=json.load(open('gpurun_out/maxn_ab_$V.json'));print(d['ms_per_step'])")"
  done
done
PHX_GEMM1_MAXN=32 timeout -k 10 1000 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/maxn_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 2 gpurun_out/maxn_tests.log; grep -E "^FAILED|^ERROR" gpurun_out/maxn_tests.log | head -20
exit $rc
