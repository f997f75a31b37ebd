# GPU: A/B of one environment knob on the default bench (alternating, 3 rounds) after the parity
# tests of the attack path.  usage: bash scripts/gpu_ab_env.sh VAR=value_b [extra bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
KV="$1"; shift
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_firstpass.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_ab.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then E=""; else E="$KV"; fi
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile "$@" > gpurun_out/ab.json 2> gpurun_out/ab.err
    rc=$?; echo "$v [$E] rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['ms_per_step'],d['value'])")"
    [ $rc -eq 0 ] || exit $rc
  done
done
