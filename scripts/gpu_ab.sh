# GPU: parity tests, then the bench line under two environment settings (A/B), no CPU leg
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error|error" gpurun_out/pytest.log | tail -5
[ $rc -eq 0 ] || exit $rc
for setting in "$@"; do
  env $setting timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile > gpurun_out/bench_ab.json 2> gpurun_out/bench_ab.err
  rc=$?; echo "[$setting] rc=$rc $(python -c 'import json;d=json.load(open("gpurun_out/bench_ab.json"));print(d["value"],d["ms_per_step"])')"
  [ $rc -eq 0 ] || exit $rc
done
