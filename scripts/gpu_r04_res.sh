# GPU: A-resident GEMM sweeps (k_gemm2r) — step parity suites, then the C2 and C4 bench A/B
# (PHX_GEMM_RES=0/1, alternating).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_bf16.py tests/test_gpu_concurrent.py \
  tests/test_gpu_deep.py -v -m gpu -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/pytest_res.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed|Error" gpurun_out/pytest_res.log | tail -40
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in 0 1; do
    PHX_GEMM_RES=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --no-secondary --steps 100 > gpurun_out/ab.json 2> gpurun_out/ab.err
    rc=$?; echo "C2 PHX_GEMM_RES=$v rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['ms_per_step'],d['value'])")"
    [ $rc -eq 0 ] || exit $rc
  done
done
for v in 0 1; do
  PHX_GEMM_RES=$v timeout -k 10 300 python bench.py --model efficientdet-d4 --dtype bf16 --image-size 1024 --batch 4 --steps 30 \
    --no-cpu-baseline --no-profile --no-secondary > gpurun_out/ab4.json 2> gpurun_out/ab4.err
  rc=$?; echo "C4 PHX_GEMM_RES=$v rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/ab4.json'));print(d['ms_per_step'],d['value'])")"
  [ $rc -eq 0 ] || exit $rc
done
