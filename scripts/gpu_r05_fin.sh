# GPU: in-launch BN finalize — step parity suites, stream-hazard checksums, C2 A/B (PHX_FIN_MAX=0 = separate launches)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_concurrent.py \
  tests/test_gpu_stream_hazard.py tests/test_gpu_deep.py -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/fin_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/fin_tests.log; grep -E "FAILED|Error|assert" gpurun_out/fin_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for x in 8192 0; do
    PHX_FIN_MAX=$x timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --no-profile > gpurun_out/fin_$x.json 2>/dev/null || exit 1
    echo "round $r PHX_FIN_MAX=$x: $(python -c "import json;d=json.load(open('gpurun_out/fin_$x.json'));print(d['ms_per_step'])")"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/finprof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-profile > gpurun_out/finprof.log 2>&1 || { tail -20 gpurun_out/finprof.log; exit 1; }
