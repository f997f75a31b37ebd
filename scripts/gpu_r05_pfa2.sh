# GPU: attacker prefetch forked at stage 6 — prefetch parity tests, then the secondary flow A/B
# (PHX_PF_FORK 0 = after the paste / 1 = at the second pass's stage 6), two rounds
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_concurrent.py > gpurun_out/pfa2_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/pfa2_tests.log; grep -E "FAILED|^E " gpurun_out/pfa2_tests.log | head; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for x in 0 1; do
    PHX_PF_FORK=$x timeout -k 10 400 python bench.py --no-cpu-baseline --no-profile --steps 100 > gpurun_out/pfa2_$x.json 2> gpurun_out/pfa2_$x.err || { tail -5 gpurun_out/pfa2_$x.err; exit 1; }
    echo "round $r PHX_PF_FORK=$x: $(python -c "import json;d=json.load(open('gpurun_out/pfa2_$x.json'));print(d['ms_per_step'], d['secondary']['ms_per_step'], d['secondary']['value'])")"
  done
done
