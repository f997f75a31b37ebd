set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|PASSED|FAILED" gpurun_out/pytest.log | tail -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --model efficientdet-d4 --image-size 1024 --batch 4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_d4.json 2> gpurun_out/bench_d4.err
rc=$?; echo "bench d4 rc=$rc"; cat gpurun_out/bench_d4.json
