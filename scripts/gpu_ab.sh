# GPU A/B: alternate `python bench.py` between libphx.so and the variant(s) in $PHX_AB (e.g.
# "libphx_swz.so"), three rounds each, then print ms/step per library.  Optional pytest first
# ($PHX_TESTS: test paths).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "${PHX_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest $PHX_TESTS -v -m gpu -p no:cacheprovider --timeout 600 --timeout-method thread \
    > gpurun_out/pytest_ab.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_ab.log | tail -20
  [ $rc -le 1 ] || exit $rc
fi
for r in 1 2 3; do
  for lib in libphx.so ${PHX_AB}; do
    PHX_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --no-profile --steps ${PHX_STEPS:-100} ${PHX_BENCH_ARGS:-} \
      > gpurun_out/ab_${lib}_$r.json 2> gpurun_out/ab_${lib}_$r.err || exit $?
    python -c "import json,sys; d=json.load(open('gpurun_out/ab_${lib}_$r.json')); print('$lib round $r', d['ms_per_step'], 'ms/step', d['value'], 'img/s')"
  done
done
