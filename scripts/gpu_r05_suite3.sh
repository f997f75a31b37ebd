# GPU: the full -m gpu suite on the wave-split-K build, then the C2 bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 600 --timeout-method thread \
  > gpurun_out/pytest_suite3.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_suite3.log; grep -E "FAILED|ERROR" gpurun_out/pytest_suite3.log | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_suite3.json 2> gpurun_out/bench_suite3.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_suite3.json; exit $rc
