# GPU: bf16 activation storage — the bf16 parity tests and the fp32 parity tests, then the C2
# (fp32) and C4 (D4 1024^2 x4 bf16) bench lines.  Stops at the first failing step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_parity.py -v -m gpu -p no:cacheprovider \
  --timeout 900 --timeout-method thread -x > gpurun_out/pytest_bf16.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed|assert" gpurun_out/pytest_bf16.log | tail -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --steps 100 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model efficientdet-d4 --dtype bf16 --image-size 1024 --batch 4 --steps 50 \
  --no-cpu-baseline --no-secondary > gpurun_out/bench_d4bf16.json 2> gpurun_out/bench_d4bf16.err
rc=$?; echo "d4 rc=$rc"; cat gpurun_out/bench_d4bf16.json; tail -3 gpurun_out/bench_d4bf16.err
exit $rc
