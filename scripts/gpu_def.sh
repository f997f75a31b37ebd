# GPU: defender parity + C5 bench line + kernel-trace summary
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_defender.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_def.log 2>&1
rc=$?; echo "pytest def rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed|Error|assert" gpurun_out/pytest_def.log | tail -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/defender_bench.py --batch 8 > gpurun_out/def_b8.json 2> gpurun_out/def_b8.err
rc=$?; echo "def b8 rc=$rc"; cat gpurun_out/def_b8.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_def -o run --output-format csv -- \
  python tools/defender_bench.py --batch 8 --steps 5 > gpurun_out/prof_def.log 2>&1
echo "rocprof def rc=$?"
