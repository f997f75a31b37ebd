# GPU: defender first-pass prefetch — the defender suites (prefetch parity included), then C5 with and
# without the prefetch (alternating, two rounds)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_defender.py tests/test_gpu_frozen_reuse.py tests/test_gpu_defender_512.py > gpurun_out/pf_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/pf_tests.log; grep -E "FAILED|^E " gpurun_out/pf_tests.log | head; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for x in no yes; do
    f=""; [ $x = no ] && f="--no-prefetch"
    timeout -k 10 300 python tools/defender_bench.py --no-cpu-baseline --no-profile $f > gpurun_out/pf_$x.json 2> gpurun_out/pf_$x.err || { tail -5 gpurun_out/pf_$x.err; exit 1; }
    echo "C5 round $r prefetch=$x: $(python -c "import json;d=json.load(open('gpurun_out/pf_$x.json'));print(d['ms_per_step'], d['value'])")"
  done
done
