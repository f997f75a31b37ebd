# GPU: the bf16 wave-split-K decision: the layer diagnosis, the bf16 parity and
# stream-hazard suites with PHX_GEMM_WSK_BF16=1, and alternating C4 A/B (0 / 1)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-wskbf}
timeout -k 10 900 python -u scripts/diag_bf16_wsk_layers.py > gpurun_out/${tag}_layers.txt 2>&1 || exit 3
tail -7 gpurun_out/${tag}_layers.txt
PHX_GEMM_WSK_BF16=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_stream_hazard.py -v -m gpu \
  -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?; echo "pytest (WSK_BF16=1) rc=$rc"; grep -E "PASSED|FAILED|ERROR" gpurun_out/${tag}_tests.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for r in 1 2; do
  for x in 0 1; do
    PHX_GEMM_WSK_BF16=$x timeout -k 10 300 python bench.py --model efficientdet-d4 --image-size 1024 --batch 4 --dtype bf16 \
      --steps 30 --no-cpu-baseline --no-secondary --no-profile > gpurun_out/${tag}_c4_$x.json 2> gpurun_out/${tag}_c4_$x.err || exit 3
    echo "round $r WSK_BF16=$x: $(python -c "import json;d=json.load(open('gpurun_out/${tag}_c4_$x.json'));print(d['ms_per_step'], d['value'])")"
  done
done
exit $rc
