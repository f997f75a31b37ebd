# GPU: kernel-trace profiles of the bench under two environment settings (no tests)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
i=0
for setting in "$@"; do
  i=$((i+1))
  env $setting timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof$i -o run --output-format csv -- \
    python bench.py --no-cpu-baseline --steps 5 --warmup 2 --no-profile > gpurun_out/prof_bench$i.log 2>&1
  rc=$?; echo "[$setting] rocprof rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
