# GPU: the A-resident GEMM with two-deep prefetch — step parity, then the C4 / C2 bench A/B:
# libphx.so (PF2) vs libphx_rpf1.so (one-deep) vs PHX_GEMM_RES=0 (the per-N-tile kernel).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_bf16.py tests/test_gpu_parity.py -k "not soft_nms" -v -m gpu \
  -p no:cacheprovider --timeout 500 --timeout-method thread > gpurun_out/pytest_respf.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed|Error" gpurun_out/pytest_respf.log | tail -20
[ $rc -eq 0 ] || exit $rc
run() {  # label, env..., then bench args
  local label=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --no-secondary $BARGS > gpurun_out/ab.json 2> gpurun_out/ab.err
  local rc=$?; echo "$label rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['ms_per_step'],d['value'])")"
  return $rc
}
BARGS="--model efficientdet-d4 --dtype bf16 --image-size 1024 --batch 4 --steps 30"
for r in 1 2; do
  run "C4 pf2" PHX_LIB=libphx.so && run "C4 pf1" PHX_LIB=libphx_rpf1.so && run "C4 res0" PHX_GEMM_RES=0 || exit 1
done
BARGS="--steps 100"
for r in 1 2; do
  run "C2 pf2" PHX_LIB=libphx.so && run "C2 pf1" PHX_LIB=libphx_rpf1.so && run "C2 res0" PHX_GEMM_RES=0 || exit 1
done
