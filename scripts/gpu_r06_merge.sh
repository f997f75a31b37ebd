# GPU: an exact rewrite against the previous build (libphx_prev.so): whole-step bit identity
# (tools/step_hash.py), alternating C2 A/B, the parity / concurrency suites on the new build and the
# launch count per step (kernel trace, one stream)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-merge}
PHX_LIB=libphx_prev.so timeout -k 10 300 python tools/step_hash.py > gpurun_out/${tag}_hash_prev.txt 2>&1 || exit 3
timeout -k 10 300 python tools/step_hash.py > gpurun_out/${tag}_hash_new.txt 2>&1 || exit 3
grep -v amdgpu.ids gpurun_out/${tag}_hash_prev.txt; grep -v amdgpu.ids gpurun_out/${tag}_hash_new.txt
for r in 1 2 3; do
  for L in libphx_prev.so libphx.so; do
    PHX_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --no-profile > gpurun_out/${tag}_$L.json 2>gpurun_out/${tag}_$L.err || exit 3
    echo "round $r $L: $(python -c "import json;d=json.load(open('gpurun_out/${tag}_$L.json'));print(d['ms_per_step'])")"
  done
done
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_concurrent.py tests/test_gpu_firstpass.py -q -m gpu \
  -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${tag}_tests.log; grep -E "^FAILED|^ERROR" gpurun_out/${tag}_tests.log | head
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash scripts/gpu_r06_kt.sh ${tag} || exit 3
exit $rc
