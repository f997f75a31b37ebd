# GPU: per-shape GEMM timings of the current planner (tools/gemm_bench, fp32 raw + statistics), a
# tile x split sweep of the deep-K D0 shapes in the BN-view and gradient-view modes, and the D0
# per-shape step profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 ./tools/gemm_bench > gpurun_out/gemm_bench_r04.txt 2>&1
rc=$?; echo "gemm_bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
GEMM_ONLY=8,10,13,15,16,18 GEMM_SWEEP=1 GEMM_MODE=1 timeout -k 10 240 ./tools/gemm_bench > gpurun_out/gemm_sweep_m1_r04.txt 2>&1
rc=$?; echo "sweep m1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
GEMM_ONLY=8,10,13,15,16,18 GEMM_SWEEP=1 GEMM_MODE=3 timeout -k 10 240 ./tools/gemm_bench > gpurun_out/gemm_sweep_m3_r04.txt 2>&1
rc=$?; echo "sweep m3 rc=$rc"; [ $rc -eq 0 ] || exit $rc
PHX_PROF_DETAIL=1 timeout -k 10 300 python tools/shape_prof.py --top 80 > gpurun_out/shapes_d0_r04.txt 2>&1
rc=$?; echo "shapes rc=$rc"; [ $rc -eq 0 ] || exit $rc
grep "^best" gpurun_out/gemm_sweep_m1_r04.txt gpurun_out/gemm_sweep_m3_r04.txt
