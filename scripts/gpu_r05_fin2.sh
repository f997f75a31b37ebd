# GPU: narrow BN finalize + in-launch finalize — step parity suites, stream hazards, C2 A/B of the two knobs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_concurrent.py \
  tests/test_gpu_stream_hazard.py tests/test_gpu_deep.py tests/test_gpu_bn_sync.py -x -v -m gpu -p no:cacheprovider \
  --timeout 300 --timeout-method thread > gpurun_out/fin2_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/fin2_tests.log; grep -E "FAILED|Error|assert" gpurun_out/fin2_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for cfg in "8192 1" "0 1" "0 0" "8192 0"; do
    set -- $cfg
    PHX_FIN_MAX=$1 PHX_FIN_NARROW=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --no-profile > gpurun_out/fin2_$1_$2.json 2>/dev/null || exit 1
    echo "round $r PHX_FIN_MAX=$1 NARROW=$2: $(python -c "import json;d=json.load(open('gpurun_out/fin2_$1_$2.json'));print(d['ms_per_step'])")"
  done
done
