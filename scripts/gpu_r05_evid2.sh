# GPU: evidence for the wave-split-K build — C2 HBM traffic (FETCH / WRITE passes), the C2 kernel-trace
# summary, and the C4 / C5 lines
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
RX='k_gemm|k_dw_|k_colred|k_bn_finalize|k_se_mlp|k_ew_gstats'
pass() {  # tag counter regex cmd...
  local tag=$1 ctr=$2 rx=$3; shift 3
  timeout -s KILL 240 rocprofv3 --pmc $ctr --kernel-include-regex "$rx" -d gpurun_out/pmc6_$tag -o run --output-format csv -- "$@" \
    > gpurun_out/pmc6_$tag.log 2>&1
  local rc=$?; echo "pmc $tag rc=$rc"; [ $rc -eq 0 ] || tail -5 gpurun_out/pmc6_$tag.log; return $rc
}
pass c2_fetch FETCH_SIZE "$RX" python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-secondary &&
pass c2_write WRITE_SIZE "$RX" python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-secondary || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_wsk -o run --output-format csv -- \
  python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-secondary > gpurun_out/prof_wsk.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model efficientdet-d4 --dtype bf16 --image-size 1024 --batch 4 --steps 50 \
  --no-cpu-baseline --no-secondary > gpurun_out/bench_d4_wsk.json 2> gpurun_out/bench_d4_wsk.err
rc=$?; echo "d4 rc=$rc"; cat gpurun_out/bench_d4_wsk.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/defender_bench.py > gpurun_out/defender_wsk.json 2> gpurun_out/defender_wsk.err
rc=$?; echo "defender rc=$rc"; cat gpurun_out/defender_wsk.json; exit $rc
