# GPU: soft-NMS parity (dense stress case, first pass), first-pass placement bench, then the fp32
# GEMM BK=32 variant (libphx_bk.so) A/B against the default build on the C2 bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_firstpass.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_nms.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_nms.log | tail -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --placement first-pass --person-bias 4.6 > gpurun_out/bench_fp.json 2> gpurun_out/bench_fp.err
rc=$?; echo "bench fp rc=$rc"; cat gpurun_out/bench_fp.json
[ $rc -eq 0 ] || exit $rc
for lib in libphx.so libphx_bk.so libphx.so libphx_bk.so; do
  PHX_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile > gpurun_out/ab.json 2> gpurun_out/ab.err
  rc=$?; echo "$lib rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['ms_per_step'],d['value'])")"
  [ $rc -eq 0 ] || exit $rc
done
