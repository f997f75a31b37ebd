# GPU: the U-Net's implicit im2col — defender parity tests (256^2, 512^2) incl. the bit-identity test
# against the column-matrix path, then the defender bench A/B (PHX_UN_GATHER=0/1, alternating).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_defender.py tests/test_gpu_defender_512.py -v -m gpu -p no:cacheprovider \
  --timeout 400 --timeout-method thread > gpurun_out/pytest_gather.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed|Error" gpurun_out/pytest_gather.log | tail -20
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in 0 1; do
    PHX_UN_GATHER=$v timeout -k 10 300 python tools/defender_bench.py --no-cpu-baseline > gpurun_out/defab.json 2> gpurun_out/defab.err
    rc=$?; echo "PHX_UN_GATHER=$v rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/defab.json'));print(d['ms_per_step'],d['value'],d['step_roofline']['breakdown_ms'].get('unet_conv'))")"
    [ $rc -eq 0 ] || exit $rc
  done
done
