# GPU: parity tests, then a rocprofv3 kernel-trace of a short bench run (summaries -> gpurun_out/prof)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -q -m gpu -p no:cacheprovider > gpurun_out/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
  python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-profile > gpurun_out/prof_bench.log 2>&1
echo "rocprof rc=$?"
