# GPU: row-store GEMM epilogue — bit-identity tests, per-shape gemm_bench (RS off / on), then the
# default bench A/B (PHX_GEMM_RS=0/1, alternating, 3 rounds).  Stops at the first failing step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_gemm_rows.py tests/test_gpu_standard_draw.py -v -m gpu -p no:cacheprovider --timeout 700 \
  --timeout-method thread > gpurun_out/pytest_rs.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed|Error|gpu vs" gpurun_out/pytest_rs.log | tail -30
[ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  PHX_GEMM_RS=$v timeout -k 10 120 tools/gemm_bench > gpurun_out/gemm_bench_rs$v.txt 2>&1
  rc=$?; echo "gemm_bench RS=$v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
paste -d'\n' gpurun_out/gemm_bench_rs0.txt gpurun_out/gemm_bench_rs1.txt | grep impl2 | head -60
bash scripts/gpu_ab_env3.sh PHX_GEMM_RS
