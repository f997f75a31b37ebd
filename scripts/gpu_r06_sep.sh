# GPU: fused separable conv — its tests, the oracle parity suites, then bench A/B (PHX_SEP=1 / 0)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-sep}
timeout -k 10 600 python -u -m pytest tests/test_gpu_sep.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -v -m gpu \
  -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${tag}_tests.log; grep -E "^FAILED|^ERROR|Error|assert" gpurun_out/${tag}_tests.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for r in 1 2; do
  for x in 1 0; do
    PHX_SEP=$x timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary > gpurun_out/${tag}_b$x.json 2> gpurun_out/${tag}_b$x.err || exit 3
    echo "round $r PHX_SEP=$x: $(python -c "import json;d=json.load(open('gpurun_out/${tag}_b$x.json'));print(d['ms_per_step'], d['value'], d['roofline']['kernel'], d['roofline']['avg_us'], d['roofline']['frac'])")"
  done
done
exit $rc
