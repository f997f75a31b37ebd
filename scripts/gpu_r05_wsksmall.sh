# GPU: wave-split-K for the few-tile unsplit GEMMs — the step parity suites, then C2 / C5 A/B of
# PHX_GEMM_WSK_SMALL 0 / 1 (alternating)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_deep.py tests/test_gpu_concurrent.py tests/test_gpu_fin.py \
  > gpurun_out/wsksmall_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/wsksmall_tests.log; grep -E "FAILED|^E " gpurun_out/wsksmall_tests.log | head; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for x in 0 1; do
    PHX_GEMM_WSK_SMALL=$x timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --no-secondary --steps 100 > gpurun_out/wsm_$x.json 2>/dev/null || exit 1
    echo "C2 round $r WSK_SMALL=$x: $(python -c "import json;d=json.load(open('gpurun_out/wsm_$x.json'));print(d['ms_per_step'])")"
  done
done
for x in 0 1; do
  PHX_GEMM_WSK_SMALL=$x timeout -k 10 300 python tools/defender_bench.py --no-cpu-baseline --no-profile > gpurun_out/wsmd_$x.json 2>/dev/null || exit 1
  echo "C5 WSK_SMALL=$x: $(python -c "import json;d=json.load(open('gpurun_out/wsmd_$x.json'));print(d['ms_per_step'])")"
done
