# GPU: parity of the attack path, then tools/gemm_bench (D0 shapes) and the default bench line x2
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_firstpass.py tests/test_gpu_deep.py tests/test_gpu_bf16.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_ab.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 tools/gemm_bench > gpurun_out/gb_stats.txt 2>&1; rc=$?; echo "gemm_bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile > gpurun_out/ab.json 2> gpurun_out/ab.err
  rc=$?; echo "bench rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['ms_per_step'],d['value'])")"
  [ $rc -eq 0 ] || exit $rc
done
