# GPU: fusion tests (PHX_XDW=1 explicitly), parity suite at the default (off), F2 kernel times
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_xdw.py tests/test_gpu_parity.py -x -v -m gpu \
  -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/xdw3_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/xdw3_tests.log; grep -E "FAILED|Error|assert" gpurun_out/xdw3_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
PHX_XDW=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/xprof3 -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-profile > gpurun_out/xprof3.log 2>&1 || { tail -20 gpurun_out/xprof3.log; exit 1; }
grep -h '"metric"' gpurun_out/xprof3.log | head -1
