# GPU: defender tests with the 1024-slice weight gradients (default build), then C5 A/B against 2048 /
# 4096 slices, then the default defender bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_defender.py tests/test_gpu_defender_512.py tests/test_gpu_defender_distributed.py -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_def.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_def.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in "" _s2k _s4k; do
    PHX_LIB=libphx$v.so timeout -k 10 300 python tools/defender_bench.py --no-cpu-baseline --no-profile --steps 50 > gpurun_out/abd.json 2> gpurun_out/abd.err
    rc=$?; echo "c5 lib$v rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/abd.json'));print(d['ms_per_step'],d['value'])")"
    [ $rc -eq 0 ] || exit $rc
  done
done
timeout -k 10 300 python tools/defender_bench.py > gpurun_out/defender_bench.json 2> gpurun_out/defender_bench.err
rc=$?; echo "defender rc=$rc"; cat gpurun_out/defender_bench.json
exit $rc
