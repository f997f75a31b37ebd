# GPU: wave-split-K GEMM (k_gemm2k) — tools/gemm_bench sweeps of the deep-K D0 shapes (raw, SE view,
# gradient view) against the cross-workgroup split, then the step parity tests that run those shapes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in ${WSK_MODES:-2 3}; do
  GEMM_ONLY=8,10,13,16,17,18 GEMM_WSK=1 GEMM_MODE=$m timeout -k 10 120 tools/gemm_bench > gpurun_out/wsk_m$m.txt 2>&1
  rc=$?; echo "wsk mode $m rc=$rc"; grep -E "^wsk" gpurun_out/wsk_m$m.txt; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_deep.py > gpurun_out/wsk_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/wsk_tests.log; grep -E "FAILED|ERROR|Error" gpurun_out/wsk_tests.log | head; exit $rc
