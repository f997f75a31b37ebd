# GPU: fused separable conv with one 32-column part per workgroup (PHX_SEP_PT=1: twice the
# workgroups, the depthwise pass repeated per part) against two (PT=2): sep_probe per level, the sep
# tests with PT=1, alternating C2 A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-seppt}
for pt in 2 1; do
  PHX_SEP_PT=$pt timeout -k 10 120 ./tools/sep_probe > gpurun_out/${tag}_probe$pt.txt 2>&1 || exit 3
  echo "PT=$pt"; grep -E "64x64|32x32" gpurun_out/${tag}_probe$pt.txt
done
PHX_SEP_PT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_sep.py -q -m gpu -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?; echo "pytest (PT=1) rc=$rc"; tail -2 gpurun_out/${tag}_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for r in 1 2 3; do
  for pt in 2 1; do
    PHX_SEP_PT=$pt timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --no-profile > gpurun_out/${tag}_b$pt.json 2>gpurun_out/${tag}_b$pt.err || exit 3
    echo "round $r PT=$pt: $(python -c "import json;d=json.load(open('gpurun_out/${tag}_b$pt.json'));print(d['ms_per_step'])")"
  done
done
exit $rc
