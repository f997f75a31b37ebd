# GPU: prefetch edge cases (mismatched batch, weight reload) and the concurrency suite
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_concurrent.py tests/test_gpu_defender.py > gpurun_out/pfa3_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/pfa3_tests.log; grep -E "FAILED|^E " gpurun_out/pfa3_tests.log | head; exit $rc
