# GPU: parity tests -> default bench line (cpu_baseline + roofline) -> rocprofv3 kernel-trace summary
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_full.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
  python bench.py --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1
echo "rocprof rc=$?"
