# GPU: the default bench line (with cpu_baseline + roofline), then the rocprofv3 kernel-trace summary of
# the same timed workload (CPU leg skipped) -> gpurun_out/full_prof
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 900 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
rc=$?
echo "bench rc=$rc"
cat gpurun_out/bench_full.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/full_prof -o run --output-format csv -- \
  python bench.py --no-cpu-baseline > gpurun_out/full_prof_bench.log 2>&1
echo "rocprof rc=$?"
