# GPU: full -m gpu suite, the C2 bench line, the C4 and C5 lines (round 6)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-r06}
timeout -k 10 1000 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${tag}_tests.log; grep -E "^FAILED|^ERROR" gpurun_out/${tag}_tests.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || exit 3
python -c "import json;d=json.load(open('gpurun_out/${tag}_bench.json'));print('C2', d['ms_per_step'], d['value'], d['roofline']['kernel'], d['roofline']['frac'], 'secondary', d['secondary']['value'], d['secondary']['steps'])"
timeout -k 10 300 python bench.py --model efficientdet-d4 --image-size 1024 --batch 4 --dtype bf16 --steps 30 --no-cpu-baseline --no-secondary > gpurun_out/${tag}_bench_d4bf16.json 2> gpurun_out/${tag}_bench_d4bf16.err || exit 3
python -c "import json;d=json.load(open('gpurun_out/${tag}_bench_d4bf16.json'));print('C4', d['ms_per_step'], d['value'])"
timeout -k 10 300 python tools/defender_bench.py > gpurun_out/${tag}_defender.json 2> gpurun_out/${tag}_defender.err || exit 3
python -c "import json;d=json.load(open('gpurun_out/${tag}_defender.json'));print('C5', d['ms_per_step'], d['value'], d['roofline'] is not None, d['cpu_baseline'] is not None)"
exit $rc
