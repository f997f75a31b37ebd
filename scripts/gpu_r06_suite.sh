# GPU: the full -m gpu suite, then the default bench line (round 6)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-r06}
timeout -k 10 1000 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${tag}_tests.log; grep -E "^FAILED|^ERROR" gpurun_out/${tag}_tests.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
rc2=$?; echo "bench rc=$rc2"; cat gpurun_out/${tag}_bench.json | cut -c1-600
exit $rc
