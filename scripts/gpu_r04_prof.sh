# GPU: default bench line + rocprofv3 kernel-trace stats of a short bench (per-kernel averages).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-x}
timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json | python -c "import json,sys;d=json.load(sys.stdin);print(d['ms_per_step'],d['value'],d['roofline']['frac'],d['roofline']['avg_us'])"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- \
  python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-secondary --no-profile > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(ls gpurun_out/prof_$TAG/*/run_kernel_stats.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(find gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/kstats_$TAG.csv; echo "stats: $f"
