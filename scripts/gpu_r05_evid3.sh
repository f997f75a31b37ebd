# GPU: round-5 closing evidence — MFMA-busy / wait counters of C2 (k_gemm2k included), the kernel
# traces of C5 with the first-pass prefetch and of the reference's placement flow
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
MF="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
RXM='k_gemm|k_dw_|k_colred|k_bn_finalize|k_se_mlp|k_ew_gstats|k_pre_nms|k_soft_nms'
timeout -s KILL 240 rocprofv3 --pmc $MF --kernel-include-regex "$RXM" -d gpurun_out/pmc7_mfma_d0 -o run --output-format csv -- \
  python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-secondary > gpurun_out/pmc7_mfma_d0.log 2>&1
rc=$?; echo "pmc mfma rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/pmc7_mfma_d0.log; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5pf -o run --output-format csv -- \
  python tools/defender_bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-profile > gpurun_out/prof_c5pf.log 2>&1
rc=$?; echo "rocprof c5 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fp -o run --output-format csv -- \
  python bench.py --placement first-pass --steps 20 --warmup 3 --no-cpu-baseline --no-secondary --no-profile > gpurun_out/prof_fp.log 2>&1
rc=$?; echo "rocprof first-pass rc=$rc"; exit $rc
