# GPU: XCD-aware tile ranges of the U-Net's small 3x3 convs (k_conv3_small) against the previous build
# (libphx_prev.so): defender steps bit for bit, the defender suites, alternating C5 A/B, the U-Net PMC
# traffic of the new build
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-unet}
PHX_LIB=libphx_prev.so timeout -k 10 300 python tools/step_hash.py --defender > gpurun_out/${tag}_hash_prev.txt 2>&1 || exit 3
timeout -k 10 300 python tools/step_hash.py --defender > gpurun_out/${tag}_hash_new.txt 2>&1 || exit 3
grep -v amdgpu.ids gpurun_out/${tag}_hash_prev.txt; grep -v amdgpu.ids gpurun_out/${tag}_hash_new.txt
timeout -k 10 700 python -u -m pytest tests/test_gpu_defender.py tests/test_gpu_defender_512.py -q -m gpu \
  -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${tag}_tests.log; grep -E "^FAILED|^ERROR" gpurun_out/${tag}_tests.log | head
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for r in 1 2 3; do
  for L in libphx_prev.so libphx.so; do
    PHX_LIB=$L timeout -k 10 200 python tools/defender_bench.py --no-cpu-baseline --no-profile > gpurun_out/${tag}_$L.json 2>gpurun_out/${tag}_$L.err || exit 3
    echo "round $r $L: $(python -c "import json;d=json.load(open('gpurun_out/${tag}_$L.json'));print(d['ms_per_step'])")"
  done
done
PMC_RX='k_conv3_small|k_gemm2|k_wgrad|k_colred64|k_un_|k_im2col|k_soft_nms' \
PMC_CMD="python tools/defender_bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile" \
  bash scripts/gpu_pmc.sh > gpurun_out/${tag}_pmc.log 2>&1 || { tail -3 gpurun_out/${tag}_pmc.log; exit 3; }
python scripts/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/${tag}_pmc_traffic_defender.json defender "python tools/defender_bench.py --steps 2 --warmup 1 (C5, round 6)" > gpurun_out/${tag}_pmc_summary.txt 2>&1 || exit 3
tail -8 gpurun_out/${tag}_pmc_summary.txt
rm -rf gpurun_out/pmc_fetch gpurun_out/pmc_write
exit $rc
