# GPU: rocprofv3 kernel trace (+ stats) of the default bench (concurrent first pass), for the timeline
# analysis (scripts/trace_step.py) and the committed kernel summary.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_conc -o run --output-format csv -- \
  python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-profile --no-secondary > gpurun_out/prof_conc.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
