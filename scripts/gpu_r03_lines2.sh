# GPU: round-3 evidence v3 — the default bench line (with the CPU baseline and the first-pass line),
# the C4 (D4 bf16 1024^2 x4) and C5 (defender) lines, each bounded by its own time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_full.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model efficientdet-d4 --dtype bf16 --image-size 1024 --batch 4 --steps 50 \
  --no-cpu-baseline --no-secondary > gpurun_out/bench_d4bf16.json 2> gpurun_out/bench_d4bf16.err
rc=$?; echo "d4 rc=$rc"; cat gpurun_out/bench_d4bf16.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/defender_bench.py > gpurun_out/defender_bench.json 2> gpurun_out/defender_bench.err
rc=$?; echo "defender rc=$rc"; cat gpurun_out/defender_bench.json
exit $rc
