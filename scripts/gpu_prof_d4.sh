# GPU: kernel-trace summary of the C4 bench (D4 1024^2 x4, bf16) and the bf16 parity tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_bf16.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed|^E  " gpurun_out/pytest_bf16.log | grep -v "where\|+  " | tail -12
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_d4 -o run --output-format csv -- \
  python bench.py --no-cpu-baseline --no-profile --model efficientdet-d4 --image-size 1024 --batch 4 --steps 5 --warmup 1 --dtype bf16 > gpurun_out/prof_d4.log 2>&1
echo "rocprof rc=$?"
