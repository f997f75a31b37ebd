# GPU: the whole -m gpu suite (verbose, per-test thread timeouts), then the default bench line and
# the first-pass-placement bench line (person_bias 4.6: real soft-NMS candidates)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest.log | tail -40
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --placement first-pass --person-bias 4.6 > gpurun_out/bench_fp.json 2> gpurun_out/bench_fp.err
rc=$?; echo "bench fp rc=$rc"; cat gpurun_out/bench_fp.json; tail -3 gpurun_out/bench_fp.err
