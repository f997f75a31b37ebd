set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu -p no:cacheprovider > gpurun_out/pytest1.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -le 1 ]; then
  timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench1.log 2>&1
  echo "bench rc=$?"
fi
