# GPU: inference-BN statistics reuse — bit-identity tests, the defender suites, C5 A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_frozen_reuse.py tests/test_gpu_defender.py tests/test_gpu_firstpass.py \
  -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/frz_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/frz_tests.log; grep -E "FAILED|Error|^E " gpurun_out/frz_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for x in 1 0; do
    PHX_FROZEN_REUSE=$x timeout -k 10 300 python tools/defender_bench.py --no-cpu-baseline --no-profile > gpurun_out/frz_$x.json 2>/dev/null || exit 1
    echo "round $r PHX_FROZEN_REUSE=$x: $(python -c "import json;d=json.load(open('gpurun_out/frz_$x.json'));print(d['ms_per_step'], d['value'])")"
  done
done
