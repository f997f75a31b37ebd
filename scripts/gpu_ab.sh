# GPU: A/B of the current build (libphx.so) against a variant ($1, e.g. libphx_pf1.so): parity of
# the current build (parity / full-size / bf16 / first-pass tests), then alternating bench lines
# (D0 C2, D4 C4 bf16) and a rocprof kernel trace of each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
ALT=${1:-libphx_pf1.so}
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_bf16.py tests/test_gpu_firstpass.py -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/pytest.log | tail -8
[ $rc -le 1 ] || exit $rc
for lib in libphx.so $ALT libphx.so $ALT; do
  for args in "" "--model efficientdet-d4 --image-size 1024 --batch 4 --steps 10 --warmup 2 --dtype bf16"; do
    PHX_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile $args > gpurun_out/ab.json 2> gpurun_out/ab.err
    rc=$?; echo "$lib [$args] rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['ms_per_step'],d['value'])")"
    [ $rc -eq 0 ] || exit $rc
  done
done
for lib in libphx.so $ALT; do
  rm -rf gpurun_out/prof_$lib
  PHX_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_$lib -o run -- python bench.py --no-cpu-baseline --no-profile --steps 10 --warmup 2 > /dev/null 2>&1
  rc=$?; echo "prof $lib rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
