# GPU: GEMM run-to-run bit identity per shape (tools/gemm_bench, modes 0 / 1 / 3), default library.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in 0 1 3; do
  for r in 1 2; do
    GEMM_MODE=$m timeout -k 10 120 ./tools/gemm_bench > gpurun_out/det.m$m.r$r.txt 2>&1
    rc=$?; echo "mode $m run $r rc=$rc nondet=$(grep -c NONDET gpurun_out/det.m$m.r$r.txt)"; [ $rc -eq 0 ] || exit $rc
  done
done
GEMM_ONLY=8,10,13,15,16,17,18 GEMM_MODE=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/gbprof -o gb -- ./tools/gemm_bench > gpurun_out/gbprof.txt 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
find gpurun_out/gbprof -name "*stats*"
