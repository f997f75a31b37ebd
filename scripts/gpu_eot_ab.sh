# GPU: EOT parity (attack step, first-pass placement, defender Masker), then the first-pass
# placement bench and the default bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_firstpass.py tests/test_gpu_fullsize.py tests/test_gpu_defender.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_eot.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_eot.log
[ $rc -eq 0 ] || exit $rc
for args in "--placement first-pass --person-bias 4.6" ""; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile $args > gpurun_out/ab.json 2> gpurun_out/ab.err
  rc=$?; echo "[$args] rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['ms_per_step'],d['value'])")"
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fp -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 5 --warmup 2 --no-profile --placement first-pass --person-bias 4.6 > gpurun_out/prof_fp.log 2>&1
echo "rocprof rc=$?"
