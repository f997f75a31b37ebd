# GPU: the full -m gpu suite (stream-hazard checker included)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 600 --timeout-method thread \
  > gpurun_out/pytest_suite.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_suite.log; grep -E "FAILED|ERROR" gpurun_out/pytest_suite.log | head
exit $rc
