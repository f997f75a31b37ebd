# GPU: the step parity suites on the default plan after the few-tile option went in (off)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_deep.py tests/test_gpu_concurrent.py tests/test_gpu_fin.py \
  > gpurun_out/recheck_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/recheck_tests.log; grep -E "FAILED|^E " gpurun_out/recheck_tests.log | head; exit $rc
