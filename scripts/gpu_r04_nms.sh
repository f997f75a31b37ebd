# GPU: soft-NMS parity (fast path, fallback, dense, first pass, defender), then the path statistics
# (PHX_NMS_STATS=1) of one defender step and one first-pass-placement attack step, then the defender
# bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_defender.py tests/test_gpu_firstpass.py -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_nms3.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|passed|failed|Error" gpurun_out/pytest_nms3.log | tail -40
[ $rc -eq 0 ] || exit $rc
PHX_NMS_STATS=1 timeout -k 10 200 python tools/defender_bench.py --steps 1 --warmup 0 > gpurun_out/nmsdbg_def.txt 2>&1
rc=$?; echo "def dbg rc=$rc"; grep "nms image" gpurun_out/nmsdbg_def.txt | head -12
[ $rc -eq 0 ] || exit $rc
PHX_NMS_STATS=1 timeout -k 10 200 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-profile --placement first-pass --person-bias 4.6 --no-secondary > gpurun_out/nmsdbg_fp.txt 2>&1
rc=$?; echo "fp dbg rc=$rc"; grep "nms image" gpurun_out/nmsdbg_fp.txt | head -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/defender_bench.py > gpurun_out/def_v3.json 2> gpurun_out/def_v3.err
rc=$?; echo "defender rc=$rc"; python -c "import json;d=json.load(open('gpurun_out/def_v3.json'));print(d['ms_per_step'],d['value'],d['step_roofline']['breakdown_ms'])"
