# GPU: secondary bench lines — C5 defender (roofline + CPU baseline) and C4 (D4 1024^2, 4 images,
# bf16) — after the defender eval test.  Stops at the first failing step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_defender.py -v -m gpu -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/pytest_def.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_def.log | tail -12
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/defender_bench.py > gpurun_out/defender_bench.json 2> gpurun_out/defender_bench.err || exit $?
cat gpurun_out/defender_bench.json
timeout -k 10 300 python bench.py --model efficientdet-d4 --dtype bf16 --image-size 1024 --batch 4 --steps 50 \
  --no-cpu-baseline > gpurun_out/bench_d4bf16.json 2> gpurun_out/bench_d4bf16.err || exit $?
cat gpurun_out/bench_d4bf16.json
