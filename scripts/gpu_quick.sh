# GPU: parity tests then a short bench line (no CPU leg) and a kernel-trace profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error|error" gpurun_out/pytest.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
  python bench.py --no-cpu-baseline --steps 5 --warmup 2 --no-profile > gpurun_out/prof_bench.log 2>&1
echo "rocprof rc=$?"
