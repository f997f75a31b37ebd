# GPU: attacker first-pass prefetch — the concurrency / first-pass / stream-hazard suites (prefetch
# parity included), then the C2 bench line (headline + the secondary first-pass flow)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_concurrent.py tests/test_gpu_firstpass.py tests/test_gpu_stream_hazard.py > gpurun_out/pfa_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/pfa_tests.log; grep -E "FAILED|^E " gpurun_out/pfa_tests.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench_pfa.json 2> gpurun_out/bench_pfa.err
rc=$?; echo "bench rc=$rc"; python -c "import json;d=json.load(open('gpurun_out/bench_pfa.json'));print(d['ms_per_step'], d['value'], d['secondary'])"; exit $rc
