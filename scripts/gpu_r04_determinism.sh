# GPU: D4 bf16 1024^2 back-to-back call identity (scripts/diag_det.py) at the default fork point, 3 runs, then
# the bf16 test suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for r in 1 2 3; do
  timeout -k 10 200 python scripts/diag_det.py efficientdet-d4 1024 bf16 2>&1 | grep -v amdgpu.ids | tail -4 | cut -c1-200
done
for r in 1 2 3; do
  timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py::test_bf16_d4_1024_four_images -q -m gpu -p no:cacheprovider \
    --timeout 250 --timeout-method thread > gpurun_out/det.log 2>&1
  echo "test round $r rc=$? $(tail -1 gpurun_out/det.log)"
done
