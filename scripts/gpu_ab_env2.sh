# GPU: parity of the attack path (incl. deep / bf16 victims), then an A/B of one environment knob on the
# D0 C2 bench and the D4 bf16 C4 bench (alternating, 2 rounds).  usage: bash scripts/gpu_ab_env2.sh VAR=value_b
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
KV="$1"
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_firstpass.py tests/test_gpu_deep.py tests/test_gpu_bf16.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_ab.log
[ $rc -eq 0 ] || exit $rc
for args in "" "--model efficientdet-d4 --image-size 1024 --batch 4 --steps 10 --warmup 2 --dtype bf16"; do
  for r in 1 2; do
    for v in A B; do
      if [ $v = A ]; then E=""; else E="$KV"; fi
      env $E timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile $args > gpurun_out/ab.json 2> gpurun_out/ab.err
      rc=$?; echo "$v [$E] [$args] rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['ms_per_step'],d['value'])")"
      [ $rc -eq 0 ] || exit $rc
    done
  done
done
