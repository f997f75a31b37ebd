# GPU: round-3 evidence of the current step — rocprofv3 kernel-trace summary of the default bench,
# MFMA / LDS-conflict counters (one PMC pass), HBM traffic (FETCH_SIZE, WRITE_SIZE: one pass each),
# the per-shape launch groups, then the C5 defender and C4 (D4 bf16) lines.  Stops at the first
# failing step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
CMD="python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-profile --no-secondary"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_d0 -o run --output-format csv -- \
  $CMD > gpurun_out/prof_d0.log 2>&1
rc=$?; echo "rocprof d0 rc=$rc"; [ $rc -eq 0 ] || exit $rc
RX='k_gemm|k_dw_|k_colred|k_bn_finalize|k_se_mlp|k_ew_gstats|k_pre_nms|k_soft_nms'
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
  --kernel-include-regex "$RX" -d gpurun_out/pmc_mfma_d0 -o run --output-format csv -- \
  python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-secondary > gpurun_out/pmc_mfma_d0.log 2>&1
rc=$?; echo "pmc mfma rc=$rc"; [ $rc -eq 0 ] || exit $rc
RX2='k_gemm|k_dw_|k_colred|k_bn_finalize|k_se_mlp|k_ew_gstats'
CMD2="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-secondary"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX2" -d gpurun_out/pmc_fetch -o run \
  --output-format csv -- $CMD2 > gpurun_out/pmc_fetch.log 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX2" -d gpurun_out/pmc_write -o run \
  --output-format csv -- $CMD2 > gpurun_out/pmc_write.log 2>&1
rc=$?; echo "write rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/shape_prof.py --top 80 > gpurun_out/shapes_d0.txt 2>&1
rc=$?; echo "d0 shapes rc=$rc"; [ $rc -eq 0 ] || exit $rc
[ -n "${PHX_NO_LINES:-}" ] && exit 0
timeout -k 10 300 python tools/defender_bench.py > gpurun_out/defender_bench.json 2> gpurun_out/defender_bench.err
rc=$?; echo "defender rc=$rc"; cat gpurun_out/defender_bench.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model efficientdet-d4 --dtype bf16 --image-size 1024 --batch 4 --steps 50 \
  --no-cpu-baseline --no-secondary > gpurun_out/bench_d4bf16.json 2> gpurun_out/bench_d4bf16.err
rc=$?; echo "d4 rc=$rc"; cat gpurun_out/bench_d4bf16.json
exit $rc
