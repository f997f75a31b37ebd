# GPU: GEMM K-chunk A/B (fp32 BK 16 -> 32, bf16 BK 32 -> 64 in libphx_bk.so): parity of the variant,
# then bench lines of both builds and rocprof traces of the variant
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
PHX_LIB=libphx_bk.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bf16.py tests/test_gpu_fullsize.py -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_bk.log 2>&1
rc=$?; echo "pytest(bk) rc=$rc"; tail -3 gpurun_out/pytest_bk.log
[ $rc -le 1 ] || exit $rc
for lib in libphx.so libphx_bk.so libphx.so libphx_bk.so; do
  for args in "" "--model efficientdet-d4 --image-size 1024 --batch 4 --steps 10 --warmup 2 --dtype bf16"; do
    PHX_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile $args > gpurun_out/ab.json 2> gpurun_out/ab.err
    rc=$?; echo "$lib [$args] rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['ms_per_step'],d['value'])")"
    [ $rc -eq 0 ] || exit $rc
  done
done
PHX_LIB=libphx_bk.so timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_bk_d0 -o run -- python bench.py --no-cpu-baseline --no-profile --steps 10 --warmup 2 > /dev/null 2>&1
echo "prof rc=$?"
