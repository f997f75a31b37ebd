# GPU: stride-2 depthwise forwards with de-interleaved window columns — step parity tests, then the
# default bench A/B (PHX_DW_DEINT=0/1, alternating, 3 rounds).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_bf16.py -k "not 1024" -v -m gpu -p no:cacheprovider --timeout 500 \
  --timeout-method thread > gpurun_out/pytest_dw.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed|Error" gpurun_out/pytest_dw.log | tail -30
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab_env3.sh PHX_DW_DEINT
