# GPU: bf16 wave-split-K with the exact-N split kept — C4 A/B (PHX_GEMM_WSK_BF16 0 / 1) and the bf16 tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
D4="--model efficientdet-d4 --image-size 1024 --batch 4 --dtype bf16"
for r in 1 2; do
  for x in 0 1; do
    PHX_GEMM_WSK_BF16=$x timeout -k 10 300 python bench.py $D4 --steps 50 --no-cpu-baseline --no-secondary --no-profile > gpurun_out/wskbf_$x.json 2> gpurun_out/wskbf_$x.err
    rc=$?; echo "C4 round $r PHX_GEMM_WSK_BF16=$x rc=$rc: $(python -c "import json;d=json.load(open('gpurun_out/wskbf_$x.json'));print(d['ms_per_step'], d['value'])")"
    [ $rc -eq 0 ] || exit $rc
  done
done
timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_bf16.py > gpurun_out/wskbf_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/wskbf_tests.log; grep -E "FAILED|^E " gpurun_out/wskbf_tests.log | head; exit $rc
