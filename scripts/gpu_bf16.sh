# GPU: bf16 parity tests, then C4 bench lines (D4 1024^2, 4 images/GPU) in fp32 and bf16
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_bf16.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed|^E  " gpurun_out/pytest_bf16.log | grep -v "where\|+  " | tail -12
[ $rc -le 1 ] || exit $rc
for dt in bf16 f32; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --model efficientdet-d4 --image-size 1024 --batch 4 --steps 10 --warmup 2 --dtype $dt > gpurun_out/bench_d4_$dt.json 2> gpurun_out/bench_d4_$dt.err
  rc=$?; echo "bench d4 $dt rc=$rc"; cat gpurun_out/bench_d4_$dt.json; tail -2 gpurun_out/bench_d4_$dt.err
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python bench.py --no-cpu-baseline --dtype bf16 > gpurun_out/bench_d0_bf16.json 2> gpurun_out/bench_d0_bf16.err
echo "bench d0 bf16 rc=$?"; cat gpurun_out/bench_d0_bf16.json
