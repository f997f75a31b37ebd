# GPU: wave-split-K with the implicit im2col — defender suites, C5 A/B (PHX_GEMM_WSK 0 / 1), mid-K sweep
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_defender.py tests/test_gpu_defender_512.py tests/test_gpu_frozen_reuse.py > gpurun_out/wskdef_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/wskdef_tests.log; grep -E "FAILED|^E " gpurun_out/wskdef_tests.log | head; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for x in 0 1; do
    PHX_GEMM_WSK=$x timeout -k 10 300 python tools/defender_bench.py --no-cpu-baseline --no-profile > gpurun_out/wskd_$x.json 2>/dev/null || exit 1
    echo "C5 round $r PHX_GEMM_WSK=$x: $(python -c "import json;d=json.load(open('gpurun_out/wskd_$x.json'));print(d['ms_per_step'], d['value'])")"
  done
done
bash scripts/gpu_r05_wsk2.sh
