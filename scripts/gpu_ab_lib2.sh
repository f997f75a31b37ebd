# GPU: alternating A/B of two in-tree builds (PHX_LIB), C2 bench without the side lines; then the
# parity suites on the new build
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
A=${1:-libphx_prev.so}; B=${2:-libphx.so}
for r in 1 2 3; do
  for L in $A $B; do
    PHX_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --no-profile > gpurun_out/ab_$L.json 2>gpurun_out/ab_$L.err || exit 3
    echo "round $r $L: $(python -c "import json;d=json.load(open('gpurun_out/ab_$L.json'));print(d['ms_per_step'])")"
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_deep.py tests/test_gpu_bf16.py -q -m gpu \
  -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/ab_tests.log; grep -E "^FAILED" gpurun_out/ab_tests.log | head
