# GPU: the whole -m gpu suite (verbose, per-test thread timeouts, heartbeat into the log), then the
# default bench line and the first-pass-placement bench line.  Stops at the first failing step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
PHX_HEARTBEAT=gpurun_out/heartbeat.log timeout -k 10 1100 python -u -m pytest tests -v -m gpu -p no:cacheprovider \
  --timeout 900 --timeout-method thread ${PHX_TESTS:-} > gpurun_out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest.log | tail -60
[ $rc -le 1 ] || exit $rc
[ -n "${PHX_NO_BENCH:-}" ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err
rc2=$?; echo "bench rc=$rc2"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
exit $(( rc > rc2 ? rc : rc2 ))
