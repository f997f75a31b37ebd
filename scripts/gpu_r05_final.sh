# GPU: round-5 evidence — the full -m gpu suite, then the C2 default bench line (CPU baseline,
# first-pass line), its rocprofv3 kernel-trace summary, and the C4 and C5 lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 600 --timeout-method thread \
  > gpurun_out/pytest_final.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_final.log; grep -E "FAILED|ERROR" gpurun_out/pytest_final.log | head
[ $rc -eq 0 ] || [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_full.json; [ $rc -eq 0 ] || [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o run --output-format csv -- \
  python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-secondary > gpurun_out/prof_final.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model efficientdet-d4 --dtype bf16 --image-size 1024 --batch 4 --steps 50 \
  --no-cpu-baseline --no-secondary > gpurun_out/bench_d4bf16.json 2> gpurun_out/bench_d4bf16.err
rc=$?; echo "d4 rc=$rc"; cat gpurun_out/bench_d4bf16.json; [ $rc -eq 0 ] || [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/defender_bench.py > gpurun_out/defender_bench.json 2> gpurun_out/defender_bench.err
rc=$?; echo "defender rc=$rc"; cat gpurun_out/defender_bench.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
D4="--model efficientdet-d4 --image-size 1024 --batch 4 --dtype bf16"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_d4 -o run --output-format csv -- \
  python bench.py $D4 --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-profile > gpurun_out/prof_d4.log 2>&1
rc=$?; echo "rocprof d4 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_def -o run --output-format csv -- \
  python tools/defender_bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-profile > gpurun_out/prof_def.log 2>&1
rc=$?; echo "rocprof def rc=$rc"; exit $rc
