# GPU: the expand -> depthwise fusion — fused vs unfused step, the oracle step tests, C2 timing A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_xdw.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -x -v -m gpu \
  -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/xdw_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/xdw_tests.log; grep -E "FAILED|Error|assert" gpurun_out/xdw_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for x in 1 0; do
    PHX_XDW=$x timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --no-profile > gpurun_out/xdw_$x.json 2>/dev/null || exit 1
    echo "round $r PHX_XDW=$x: $(python -c "import json;d=json.load(open('gpurun_out/xdw_$x.json'));print(d['ms_per_step'], d['config']['workspace_gb_per_gpu'])")"
  done
done
