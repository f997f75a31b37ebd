# GPU: fusion on/off vs the oracle for D1/D0 drop-connect steps, the remaining parity tests, C2 A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/diag_xdw_dc.py efficientdet-d1 > gpurun_out/xdw_dc.log 2>&1 || { tail -20 gpurun_out/xdw_dc.log; exit 1; }
timeout -k 10 300 python -u scripts/diag_xdw_dc.py efficientdet-d0 >> gpurun_out/xdw_dc.log 2>&1 || { tail -20 gpurun_out/xdw_dc.log; exit 1; }
cat gpurun_out/xdw_dc.log | grep PHX_XDW
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v -m gpu --deselect tests/test_gpu_parity.py::test_drop_connect_step_matches_oracle \
  -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/xdw_tests2.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/xdw_tests2.log; grep -E "FAILED|Error|assert" gpurun_out/xdw_tests2.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for r in 1 2; do
  for x in 1 0; do
    PHX_XDW=$x timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --no-profile > gpurun_out/xdw_$x.json 2>/dev/null || exit 1
    echo "round $r PHX_XDW=$x: $(python -c "import json;d=json.load(open('gpurun_out/xdw_$x.json'));print(d['ms_per_step'], d['config']['workspace_gb_per_gpu'])")"
  done
done
