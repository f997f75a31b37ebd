# GPU: closing run on HEAD — the full -m gpu suite, the default bench line (CPU baseline and the
# secondary first-pass flow included), and smoke()
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 600 --timeout-method thread \
  > gpurun_out/pytest_final2.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_final2.log; grep -E "FAILED|ERROR" gpurun_out/pytest_final2.log | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_final2.json 2> gpurun_out/bench_final2.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_final2.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final2.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke_final2.log; exit $rc
