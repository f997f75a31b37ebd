# GPU: MFMA-busy / wait-state counters of the GEMM and depthwise kernels (one PMC pass, kernel-trace
# only; 7 SQ + 1 GRBM counters fit one pass, MI355X_MICROARCH.md "rocprofv3 PMC slots")
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
RX='k_gemm|k_dw_|k_colred|k_bn_finalize|k_se_mlp|k_ew_gstats|k_pre_nms|k_soft_nms'
for args in "" "--model efficientdet-d4 --image-size 1024 --batch 4 --dtype bf16"; do
  tag=$( [ -z "$args" ] && echo d0 || echo d4bf16 )
  timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
    --kernel-include-regex "$RX" -d gpurun_out/pmc_mfma_$tag -o run --output-format csv -- \
    python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile $args > gpurun_out/pmc_mfma_$tag.log 2>&1
  rc=$?; echo "pmc $tag rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/pmc_mfma_$tag.log; exit $rc; }
done
