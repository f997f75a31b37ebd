# GPU (round 6, closing): the full -m gpu suite, smoke(), the default C2 bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-r06f}
timeout -k 10 1000 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${tag}_tests.log; grep -E "^FAILED|^ERROR" gpurun_out/${tag}_tests.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || { tail -5 gpurun_out/${tag}_smoke.log; exit 3; }
tail -2 gpurun_out/${tag}_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || exit 3
python -c "import json;d=json.load(open('gpurun_out/${tag}_bench.json'));print('C2', d['ms_per_step'], d['value'], d['roofline']['kernel'], d['roofline']['avg_us'], d['roofline']['frac'], 'secondary', d['secondary']['value'], d['secondary']['steps'], 'cpu', d['cpu_baseline']['value'])"
exit $rc
