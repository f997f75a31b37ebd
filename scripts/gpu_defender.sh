# GPU: defender parity (tests/test_gpu_defender.py), then the attack-step parity tests that share
# the generalised EOT kernels
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_defender.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_def.log 2>&1
rc=$?; echo "pytest def rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed|Error|assert" gpurun_out/pytest_def.log | tail -30
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_firstpass.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_att.log 2>&1
rc=$?; echo "pytest att rc=$rc"; tail -3 gpurun_out/pytest_att.log
