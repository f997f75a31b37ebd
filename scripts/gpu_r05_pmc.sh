# GPU: round-5 PMC evidence, one counter group per pass, kernel-trace only (MI355X_MICROARCH.md:
# FETCH_SIZE and WRITE_SIZE in separate passes; <= 8 SQ counters per pass):
#   C2 (default bench), C4 (D4 bf16 1024^2 x4) and C5 (defender) HBM traffic;
#   MFMA-busy / wait / LDS-conflict counters of C2 and C4.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
RX='k_gemm|k_dw_|k_colred|k_bn_finalize|k_se_mlp|k_ew_gstats'
RXD='k_conv3_small|k_gemm2|k_im2col|k_wgrad|k_colred64|k_un_|k_soft_nms'
D4="--model efficientdet-d4 --image-size 1024 --batch 4 --dtype bf16"
pass() {  # tag counter regex cmd...
  local tag=$1 ctr=$2 rx=$3; shift 3
  timeout -s KILL 240 rocprofv3 --pmc $ctr --kernel-include-regex "$rx" -d gpurun_out/pmc5_$tag -o run --output-format csv -- "$@" \
    > gpurun_out/pmc5_$tag.log 2>&1
  local rc=$?; echo "pmc $tag rc=$rc"; [ $rc -eq 0 ] || tail -5 gpurun_out/pmc5_$tag.log; return $rc
}
pass c2_fetch FETCH_SIZE "$RX" python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-secondary &&
pass c2_write WRITE_SIZE "$RX" python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-secondary &&
pass c4_fetch FETCH_SIZE "$RX" python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-secondary $D4 &&
pass c4_write WRITE_SIZE "$RX" python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-secondary $D4 &&
pass c5_fetch FETCH_SIZE "$RXD" python tools/defender_bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile &&
pass c5_write WRITE_SIZE "$RXD" python tools/defender_bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile || exit 1
MF="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
RXM='k_gemm|k_dw_|k_colred|k_bn_finalize|k_se_mlp|k_ew_gstats|k_pre_nms|k_soft_nms'
pass mfma_d0 "$MF" "$RXM" python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-secondary &&
pass mfma_d4 "$MF" "$RXM" python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-secondary $D4
